"""Sensor contract tests: filter policy, data_t ABI, chain tracker, prompt bytes."""
import random

import pytest
from hypothesis import given, settings, strategies as st

from chronos.native import sensor_lib
from chronos.sensor import abi, filters, render
from chronos.sensor.chain import ChainTracker, NativeChainTracker, TrackerConfig
from chronos.sensor.prompt import build_prompt, prompt_prefix
from chronos.sensor.replay import SCREENSHOT_CHAINS, SyntheticTelemetry, TelemetryConfig, attack_chain_records

# (path, dropped-by-reference-policy) — chronos_sensor.py:76-92
FILTER_TABLE = [
    ("/lib/x86_64-linux-gnu/libc.so.6", True), ("/lib", True), ("/li", False), ("/usr/lib/locale/locale-archive", True),
    ("/usr/share/zoneinfo/UTC", True), ("/etc/ssl/certs/ca.crt", True), ("/etc/fonts/fonts.conf", True),
    ("/etc/hostname", True), ("/etc/hosts", True), ("/etc/host", True), ("/etc/hos", False),
    ("/dev/null", True), ("/dev", False), ("/proc/self/maps", True), ("/proc", False),
    ("/home/u/a.so", True), ("so", False), (".so", True), ("/x/.cache", True), ("/x/y.mo", True),
    ("/etc/resolv.conf", True), ("/x/c.crt", True), ("/home/kali/.curlrc", True),
    ("/home/kali/.config/curlrc", False), ("/etc/localtime", False), ("/tmp/malware.bin", False), ("", False),
    ("/tmp/" + "a" * 300 + ".so", False),  # truncated at 255 bytes: the suffix is cut off
    ("/tmp/" + "a" * 247 + ".so", True),    # exactly 255 bytes long
]


@pytest.mark.parametrize("path,dropped", FILTER_TABLE)
def test_filter_table_python_and_native(path, dropped):
    assert filters.open_is_noise(path) == dropped
    assert sensor_lib().open_is_noise(path) == dropped


def test_strict_filter_adds_q9_cases():
    lib = sensor_lib()
    for p in ("/etc/localtime", "/home/kali/.config/curlrc"):
        assert not lib.open_is_noise(p) and lib.open_is_noise(p, True)
        assert filters.open_is_noise(p, strict=True)


@settings(max_examples=300, deadline=None)
@given(st.text(alphabet="/abcdehilnoprstuvx.-_ ", max_size=40))
def test_filter_native_matches_python(path):
    assert sensor_lib().open_is_noise(path) == filters.open_is_noise(path)


def test_record_abi_roundtrip():
    assert abi.RECORD_SIZE == 288 == sensor_lib().RECORD_SIZE
    r = abi.encode(7, "x" * 40, "/p" * 200, "EXECUTION")
    assert len(r) == 288
    ev = abi.decode(r)
    assert ev.pid == 7 and ev.comm == b"x" * 15 and len(ev.argv) == 255 and ev.type == b"EXECUTION"
    assert r == sensor_lib().encode_record(7, "x" * 40, "/p" * 200, "EXECUTION")
    (pid, comm, argv, typ), = sensor_lib().decode_records(r)
    assert (pid, comm, argv, typ) == (ev.pid, ev.comm, ev.argv, ev.type)


@pytest.mark.parametrize("impl", [ChainTracker, NativeChainTracker])
@pytest.mark.parametrize("order", ["screenshot", "time"])
def test_attack_chain_replay_reproduces_screenshot(impl, order):
    out = impl().feed_records(attack_chain_records(order), kernel_filter=True)
    got = [(t.pid, t.history) for t in out]
    if order == "screenshot":
        assert got == SCREENSHOT_CHAINS
    else:
        assert sorted(got) == sorted(SCREENSHOT_CHAINS)


def test_tracker_semantics():
    t = ChainTracker()
    assert t.feed_event(1, b"bash", b"curl", b"EXEC") is None            # trigger but chain too short
    trig = t.feed_event(1, b"curl", b"/tmp/x", b"OPEN")
    assert trig.history == ["[EXEC] bash -> curl", "[OPEN] curl -> /tmp/x"] and t.chain(1) == []
    assert t.feed_event(2, b"python3", b"curl", b"EXEC") is None and t.num_pids() == 1  # ignored comm (Q6)
    assert t.feed_event(3, b"\xff", b"x", b"OPEN") is None                # bad utf-8 dropped (Q12)
    t.feed_event(4, b"rsync", b"/a", b"EXEC")
    assert t.feed_event(4, b"rsync", b"/b", b"OPEN") is not None          # `nc` substring of rsync (Q5)
    w = ChainTracker(TrackerConfig(word_triggers=True))
    w.feed_event(4, b"rsync", b"/a", b"EXEC")
    assert w.feed_event(4, b"rsync", b"/b", b"OPEN") is None
    w.feed_event(5, b"sh", b"/tmp/a", b"OPEN")
    assert w.feed_event(5, b"sh", b"/usr/bin/nc", b"EXEC") is not None


def test_bounded_memory_fix():
    for impl in (ChainTracker, NativeChainTracker):
        t = impl(TrackerConfig(max_chain=3, max_pids=2))
        for i in range(10):
            t.feed_event(1, b"a", f"/f{i}".encode(), b"OPEN")
        assert t.chain(1) == ["[OPEN] a -> /f7", "[OPEN] a -> /f8", "[OPEN] a -> /f9"]
        t.feed_event(2, b"a", b"/x", b"OPEN")
        t.feed_event(3, b"a", b"/y", b"OPEN")
        assert t.num_pids() == 2 and t.chain(1) == []


@pytest.mark.parametrize("word", [False, True])
def test_native_tracker_equals_python_on_synthetic_fleet(word):
    cfg = TrackerConfig(word_triggers=word)
    for sensor in range(4):
        recs = SyntheticTelemetry(TelemetryConfig(seed=3), sensor_id=sensor).records(400)
        a = ChainTracker(cfg).feed_records(recs, kernel_filter=True)
        b = NativeChainTracker(cfg).feed_records(recs, kernel_filter=True)
        assert [(x.pid, x.history) for x in a] == [(x.pid, x.history) for x in b]
        assert len(a) > 20


def test_prompt_golden_bytes():
    hist = SCREENSHOT_CHAINS[0][1]
    p = build_prompt(hist)
    assert len(p) == 299
    assert p.startswith(prompt_prefix())
    expected = ("\n    Analyze this sequence. Return JSON ONLY.\n    Sequence: " + str(hist) +
                "\n    Context: 'curl' -> 'chmod' -> 'exec' is a Dropper.\n    Format: {\"risk_score\": <0-10>, "
                "\"verdict\": \"<SAFE/MALICIOUS>\", \"reason\": \"<Short Explanation>\"}\n    ")
    assert p == expected
    # quotes inside events switch Python's repr to double quotes, exactly like str(list) in the reference
    assert "\"[OPEN] a -> it's\"" in build_prompt(["[OPEN] a -> it's"])


def test_render_lines_match_reference():
    assert render.verdict_lines({"risk_score": 8, "verdict": "MALICIOUS", "reason": "r"}) == [
        "\033[91m    ==> ALERT: MALICIOUS (Risk 8)\033[0m", "    ==> REASON: r"]
    err = {"risk_score": 0, "verdict": "ERROR", "reason": "timeout"}
    assert render.verdict_lines(err)[0] == "\033[92m    ==> CLEAN: ERROR (Risk 0)\033[0m"  # Q2 in compat mode
    assert "ERROR" in render.verdict_lines(err, distinct_errors=True)[0]
    assert render.chain_lines(5, ["a"]) == ["\n[!] CAPTURED KILL CHAIN (PID 5):", "    a"]
    assert render.is_alert({"risk_score": "9"}) and not render.is_alert({"risk_score": "high"})

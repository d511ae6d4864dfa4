"""Operator console output (reference chronos_sensor.py:100,108,143-155,159).

Compat mode reproduces the reference lines byte for byte, including quirk Q2 (an ERROR verdict has risk 0 and is
printed as a green CLEAN line).  ``distinct_errors=True`` prints ERROR verdicts in yellow as ``ERROR`` instead.
A non-numeric ``risk_score`` (quirk Q11: the reference raises inside the perf callback) is treated as 0 here.
"""
from __future__ import annotations

import sys
from typing import Sequence, TextIO

RED = "\033[91m"
GREEN = "\033[92m"
YELLOW = "\033[93m"
RESET = "\033[0m"
ALERT_THRESHOLD = 5


def banner_connect(host: str) -> str:
    return f"[+] CHRONOS: Connecting to Brain at {host}..."


def banner_live() -> str:
    return "[+] CHRONOS: LIVE. Stateful Monitoring Active."


def chain_lines(pid: int, history: Sequence[str]) -> list[str]:
    return [f"\n[!] CAPTURED KILL CHAIN (PID {pid}):"] + [f"    {step}" for step in history]


def waiting_line(pid: int) -> str:
    return f"    [?] Analyzing Behavioral Chain for PID {pid} (Waiting for AI)..."


def risk_of(result: dict) -> float:
    score = result.get("risk_score", 0)
    if isinstance(score, bool):
        return int(score)
    if isinstance(score, (int, float)):
        return score
    try:
        return float(score)
    except (TypeError, ValueError):
        return 0


def is_alert(result: dict) -> bool:
    return risk_of(result) > ALERT_THRESHOLD


def verdict_lines(result: dict, distinct_errors: bool = False) -> list[str]:
    score = result.get("risk_score", 0)
    verdict = result.get("verdict")
    reason = result.get("reason")
    if distinct_errors and verdict == "ERROR":
        return [f"{YELLOW}    ==> ERROR: Brain unavailable (Risk {score}){RESET}", f"    ==> REASON: {reason}"]
    if is_alert(result):
        return [f"{RED}    ==> ALERT: {verdict} (Risk {score}){RESET}", f"    ==> REASON: {reason}"]
    return [f"{GREEN}    ==> CLEAN: {verdict} (Risk {score}){RESET}", f"    ==> REASON: {reason}"]


def emit(lines: Sequence[str], out: TextIO | None = None) -> None:
    out = out or sys.stdout
    for ln in lines:
        print(ln, file=out)
    out.flush()

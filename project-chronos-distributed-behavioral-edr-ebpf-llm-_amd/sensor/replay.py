"""Event sources that need no kernel: attack-chain replay, synthetic telemetry, and raw replay files.

* :func:`attack_chain_records` replays what the kprobes see while ``attack_chain.sh`` runs (reference
  attack_chain.sh:1-16 + SURVEY.md §3.4), *before* the in-kernel filter, as 288-byte ``data_t`` records.  Fed through
  the filter + tracker it yields exactly the four chains of the reference screenshot (PIDs 2769, 2780, 2779, 2769).
* :class:`SyntheticTelemetry` generates fleet telemetry from many sensors: benign process trees (editors, builds,
  package managers, shells, log readers), filesystem noise that the kernel filter must drop, ignored comms, and
  MITRE ATT&CK-style chains (T1105 dropper, T1059 reverse shell, T1003 credential access, T1053 persistence,
  T1082 discovery).  Deterministic for a given seed.
* Replay files are a plain concatenation of ``data_t`` records (``.chronos``), so a live capture can be replayed.
"""
from __future__ import annotations

import os
import random
from dataclasses import dataclass
from typing import Iterator

from . import abi
from .chain import ChainTracker, NativeChainTracker, TrackerConfig, Trigger


def _r(pid, comm, argv, t):
    return abi.encode(pid, comm, argv, t)


def attack_chain_records(order: str = "screenshot", user: str = "kali") -> bytes:
    """Raw kprobe stream of one ``attack_chain.sh`` run.

    ``order="screenshot"`` emits the per-process groups in the order the reference drained its per-CPU perf rings
    after the blocking Brain call (2769, 2780, 2779, then 2769's curl opens); ``"time"`` is wall-clock order.
    """
    sh, curl_pid, chmod_pid, cat_pid = "attack_chain.sh", 2769, 2779, 2780
    home = f"/home/{user}"
    g_curl_spawn = [
        _r(curl_pid, sh, "/tmp/malware.bin", "OPEN"),          # `> /tmp/malware.bin` redirect in the child
        _r(curl_pid, sh, "curl", "EXEC"),                       # pre-exec comm is still the script
    ]
    g_curl_run = [
        _r(curl_pid, "curl", "/etc/ld.so.cache", "OPEN"),       # noise (.cache)
        _r(curl_pid, "curl", "/lib/x86_64-linux-gnu/libcurl.so.4", "OPEN"),
        _r(curl_pid, "curl", "/usr/lib/ssl/openssl.cnf", "OPEN"),
        _r(curl_pid, "curl", "/etc/ssl/certs/ca-certificates.crt", "OPEN"),
        _r(curl_pid, "curl", "/etc/localtime", "OPEN"),
        _r(curl_pid, "curl", f"{home}/.config/curlrc", "OPEN"),  # `.curlrc` suffix misses this one (Q9)
        _r(curl_pid, "curl", "/etc/hosts", "OPEN"),
        _r(curl_pid, "curl", "/etc/resolv.conf", "OPEN"),
    ]
    g_chmod = [
        _r(chmod_pid, sh, "chmod", "EXEC"),
        _r(chmod_pid, "chmod", "/etc/ld.so.cache", "OPEN"),
        _r(chmod_pid, "chmod", "/lib/x86_64-linux-gnu/libc.so.6", "OPEN"),
        _r(chmod_pid, "chmod", "", "OPEN"),                      # unreadable user page at entry (Q10)
    ]
    g_cat = [
        _r(cat_pid, sh, "/dev/null", "OPEN"),                   # `> /dev/null` redirect: dropped in kernel
        _r(cat_pid, sh, "cat", "EXEC"),
        _r(cat_pid, "cat", "/etc/ld.so.cache", "OPEN"),
        _r(cat_pid, "cat", "/usr/lib/locale/locale-archive", "OPEN"),
        _r(cat_pid, "cat", "/tmp/malware.bin", "OPEN"),
    ]
    noise = [_r(2701, "python3", "/tmp/malware.bin", "OPEN"), _r(2702, "code", "/tmp/x", "OPEN")]
    if order == "screenshot":
        groups = [g_curl_spawn, g_cat, g_chmod, g_curl_run, noise]
    elif order == "time":
        groups = [g_curl_spawn, g_curl_run, g_chmod, g_cat, noise]
    else:
        raise ValueError(order)
    return b"".join(r for g in groups for r in g)


SCREENSHOT_CHAINS = [
    (2769, ["[OPEN] attack_chain.sh -> /tmp/malware.bin", "[EXEC] attack_chain.sh -> curl"]),
    (2780, ["[EXEC] attack_chain.sh -> cat", "[OPEN] cat -> /tmp/malware.bin"]),
    (2779, ["[EXEC] attack_chain.sh -> chmod", "[OPEN] chmod -> "]),
    (2769, ["[OPEN] curl -> /etc/localtime", "[OPEN] curl -> /home/kali/.config/curlrc"]),
]


def write_replay(path: str, records: bytes) -> None:
    with open(path, "wb") as f:
        f.write(records)


def read_replay(path: str) -> bytes:
    with open(path, "rb") as f:
        data = f.read()
    if len(data) % abi.RECORD_SIZE:
        raise ValueError(f"{path}: size {len(data)} is not a multiple of {abi.RECORD_SIZE}")
    return data


# ----------------------------------------------------------------------------------------------------------------
# Synthetic fleet telemetry
# ----------------------------------------------------------------------------------------------------------------
_USERS = ["alice", "bob", "svc", "root", "kali", "deploy"]
_WORDS = ["report", "data", "notes", "backup", "build", "cache", "output", "config", "main", "index", "app",
          "server", "client", "test", "tmp", "log", "db", "secret", "keys", "payload", "update", "stage"]
_EXTS = [".txt", ".log", ".json", ".csv", ".py", ".c", ".md", ".bin", ".sh", ".tar.gz", ".yaml", ".db"]
_HOSTS = ["10.0.3.7", "198.51.100.23", "203.0.113.9", "update.example.net", "cdn.example.org", "192.0.2.44"]


@dataclass
class TelemetryConfig:
    seed: int = 0
    attack_rate: float = 0.35   # fraction of process trees that are attack chains
    noise_per_proc: tuple[int, int] = (1, 6)   # kernel-filtered opens per process
    pid_base: int = 1000


class SyntheticTelemetry:
    def __init__(self, cfg: TelemetryConfig | None = None, sensor_id: int = 0):
        self.cfg = cfg or TelemetryConfig()
        self.rng = random.Random((self.cfg.seed << 20) ^ sensor_id)
        self.next_pid = self.cfg.pid_base + 7919 * sensor_id % 100000

    def _pid(self) -> int:
        self.next_pid += self.rng.randint(1, 17)
        return self.next_pid

    def _file(self, user: str) -> str:
        # a random 24-bit hex tag per file: fleet telemetry rarely repeats exact paths, and a low-entropy generator
        # would make the Brain's prefix cache look better than it is on real chains
        r = self.rng
        d = r.choice([f"/home/{user}", f"/home/{user}/src", "/tmp", "/var/tmp", "/opt/app", f"/home/{user}/Downloads"])
        return f"{d}/{r.choice(_WORDS)}_{r.getrandbits(24):06x}{r.choice(_EXTS)}"

    def _noise(self, pid: int, comm: str) -> list[bytes]:
        r = self.rng
        pool = ["/etc/ld.so.cache", "/lib/x86_64-linux-gnu/libc.so.6", "/usr/lib/locale/locale-archive",
                "/usr/share/zoneinfo/UTC", "/etc/nsswitch.conf", "/proc/self/status", "/dev/null", "/dev/tty",
                "/usr/lib/x86_64-linux-gnu/gconv/gconv-modules.cache", "/etc/ssl/openssl.cnf",
                "/usr/share/locale/en/LC_MESSAGES/coreutils.mo", "/etc/host.conf", "/etc/fonts/fonts.conf"]
        return [_r(pid, comm, r.choice(pool), "OPEN") for _ in range(r.randint(*self.cfg.noise_per_proc))]

    def _benign(self) -> list[bytes]:
        r, u = self.rng, self.rng.choice(_USERS)
        parent = r.choice(["bash", "zsh", "sshd", "cron", "systemd", "make", "tmux: server"])
        kind = r.randrange(7)
        pid = self._pid()
        out: list[bytes] = []
        if kind == 0:      # editor session
            out += [_r(pid, parent, "vim", "EXEC")] + self._noise(pid, "vim")
            out += [_r(pid, "vim", self._file(u), "OPEN") for _ in range(r.randint(1, 3))]
        elif kind == 1:    # compiler
            out += [_r(pid, "make", "gcc", "EXEC"), _r(pid, "gcc", self._file(u), "OPEN")] + self._noise(pid, "gcc")
        elif kind == 2:    # log reading (trips the `cat` trigger: benign positive for the Brain)
            out += [_r(pid, parent, "cat", "EXEC")] + self._noise(pid, "cat")
            out += [_r(pid, "cat", r.choice(["/var/log/syslog", "/var/log/auth.log", self._file(u)]), "OPEN")]
        elif kind == 3:    # package manager
            out += [_r(pid, parent, "apt-get", "EXEC")] + self._noise(pid, "apt-get")
            out += [_r(pid, "apt-get", "/var/lib/dpkg/status", "OPEN"), _r(pid, "apt-get", "/var/cache/apt/pkgcache.bin", "OPEN")]
        elif kind == 4:    # ignored tooling
            comm = r.choice(["python3", "node", "git", "code", "chrome"])
            out += [_r(pid, comm, self._file(u), "OPEN") for _ in range(r.randint(1, 4))]
        elif kind == 5:    # shell script
            out += [_r(pid, parent, "bash", "EXEC")] + self._noise(pid, "bash")
            out += [_r(pid, "bash", self._file(u), "OPEN"), _r(pid, "bash", "ls", "EXEC")]
        else:              # rsync backup (trips `nc` as a substring: quirk Q5)
            out += [_r(pid, "cron", "rsync", "EXEC")] + self._noise(pid, "rsync")
            out += [_r(pid, "rsync", self._file(u), "OPEN"), _r(pid, "rsync", f"/backup/{r.choice(_WORDS)}.tar", "OPEN")]
        return out

    def _attack(self) -> list[bytes]:
        r, u = self.rng, self.rng.choice(_USERS)
        parent = r.choice(["bash", "sh", "update.sh", "attack_chain.sh", "cron", "apache2"])
        kind = r.randrange(5)
        out: list[bytes] = []
        drop = f"/tmp/{r.choice(_WORDS)}{r.getrandbits(20):05x}{r.choice(['.bin', '', '.sh', '.elf'])}"
        if kind == 0:      # T1105 ingress tool transfer + execution
            p1, p2, p3 = self._pid(), self._pid(), self._pid()
            tool = r.choice(["curl", "wget"])
            out += [_r(p1, parent, drop, "OPEN"), _r(p1, parent, tool, "EXEC")] + self._noise(p1, tool)
            out += [_r(p1, tool, "/etc/localtime", "OPEN"), _r(p1, tool, f"/home/{u}/.config/{tool}rc", "OPEN")]
            out += [_r(p2, parent, "chmod", "EXEC")] + self._noise(p2, "chmod") + [_r(p2, "chmod", drop, "OPEN")]
            out += [_r(p3, parent, drop, "EXEC"), _r(p3, drop.rsplit("/", 1)[1][:15], "/etc/passwd", "OPEN")]
        elif kind == 1:    # T1059 reverse shell
            p = self._pid()
            out += [_r(p, parent, "bash", "EXEC"), _r(p, "bash", "/dev/tcp/" + r.choice(_HOSTS) + "/4444", "OPEN"),
                    _r(p, "bash", "nc", "EXEC"), _r(p, "nc", "/bin/sh", "OPEN")]
        elif kind == 2:    # T1003 credential access
            p = self._pid()
            out += [_r(p, parent, "cat", "EXEC")] + self._noise(p, "cat")
            out += [_r(p, "cat", f, "OPEN") for f in r.sample(["/etc/shadow", "/etc/passwd", f"/home/{u}/.ssh/id_rsa",
                                                                 "/root/.bash_history", "/etc/sudoers"], 2)]
        elif kind == 3:    # T1053 persistence via cron
            p1, p2 = self._pid(), self._pid()
            out += [_r(p1, parent, "/etc/cron.d/" + r.choice(_WORDS), "OPEN"), _r(p1, parent, "crontab", "EXEC")]
            out += [_r(p2, parent, "chmod", "EXEC"), _r(p2, "chmod", "/etc/cron.d/" + r.choice(_WORDS), "OPEN")]
        else:              # T1082 discovery then exfil
            p = self._pid()
            out += [_r(p, parent, "uname", "EXEC"), _r(p, "uname", "/etc/os-release", "OPEN"),
                    _r(p, parent, "curl", "EXEC"), _r(p, "curl", self._file(u), "OPEN")]
        return out

    def records(self, n_procs: int) -> bytes:
        buf = []
        for _ in range(n_procs):
            buf += self._attack() if self.rng.random() < self.cfg.attack_rate else self._benign()
        return b"".join(buf)


def synthetic_chains(n: int, seed: int = 0, sensors: int = 16, native: bool = True,
                     tracker_cfg: TrackerConfig | None = None) -> list[Trigger]:
    """Run synthetic fleet telemetry through the kernel filter + chain tracker until ``n`` chains fire."""
    out: list[Trigger] = []
    gens = [SyntheticTelemetry(TelemetryConfig(seed=seed), sensor_id=s) for s in range(sensors)]
    trackers = [(NativeChainTracker if native else ChainTracker)(tracker_cfg) for _ in range(sensors)]
    while len(out) < n:
        for g, t in zip(gens, trackers):
            out += t.feed_records(g.records(8), kernel_filter=True)
            if len(out) >= n:
                break
    return out[:n]


def iter_replay_dir(path: str) -> Iterator[bytes]:
    for name in sorted(os.listdir(path)):
        if name.endswith(".chronos"):
            yield read_replay(os.path.join(path, name))

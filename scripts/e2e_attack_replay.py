"""End-to-end CHRONOS: attack_chain.sh replay (and optional synthetic fleet load) -> sensor -> REST -> Brain -> verdicts.

BASELINE config 1 ("attack_chain.sh replay -> Llama-3 via Ollama REST"): the Brain is started as a separate server
process exactly like ``ollama serve`` (README.md:57-62), the sensor runs its reference loop against it
(chronos_sensor.py:159-163 semantics over the replayed 288-byte records) and prints the reference console output.

  python scripts/e2e_attack_replay.py --model llama3-8b --device cuda          # on an MI355X
  python scripts/e2e_attack_replay.py --model tiny --device cpu --fleet 32      # plumbing check, no GPU
"""
from __future__ import annotations

import argparse
import os
import socket
import subprocess
import sys
import time

import requests

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="tiny")
    ap.add_argument("--device", default="cpu")
    ap.add_argument("--port", type=int, default=0)
    ap.add_argument("--fleet", type=int, default=0, help="also analyse N synthetic fleet chains, async")
    ap.add_argument("--inflight", type=int, default=256)
    ap.add_argument("--max-slots", type=int, default=256)
    ap.add_argument("--startup-timeout", type=float, default=600)
    a = ap.parse_args(argv)
    port = a.port or free_port()
    env = dict(os.environ, PYTHONPATH=REPO + os.pathsep + os.environ.get("PYTHONPATH", ""))
    srv = subprocess.Popen([sys.executable, "-m", "chronos.brain.api", "--host", "127.0.0.1", "--port", str(port),
                            "--model", a.model, "--device", a.device, "--max-slots", str(a.max_slots),
                            "--max-model-len", "1024"], cwd=REPO, env=env)
    try:
        t0 = time.time()
        while True:
            try:
                if requests.get(f"http://127.0.0.1:{port}/healthz", timeout=2).status_code == 200:
                    break
            except requests.RequestException:
                pass
            if srv.poll() is not None or time.time() - t0 > a.startup_timeout:
                print("Brain failed to start", file=sys.stderr)
                return 1
            time.sleep(1)
        print(f"[e2e] Brain up after {time.time() - t0:.1f}s", file=sys.stderr)
        from chronos.sensor.main import run

        rc = run(["--brain", f"127.0.0.1:{port}", "--source", "attack", "--schema"])
        if rc == 0 and a.fleet:
            rc = run(["--brain", f"127.0.0.1:{port}", "--source", f"synthetic:{a.fleet}", "--schema",
                      "--async", str(a.inflight)])
        print(requests.get(f"http://127.0.0.1:{port}/metrics", timeout=5).text.split("# TYPE chronos_verdict")[0],
              file=sys.stderr)
        return rc
    finally:
        srv.terminate()
        try:
            srv.wait(timeout=30)
        except subprocess.TimeoutExpired:
            srv.kill()


if __name__ == "__main__":
    sys.exit(main())

"""Brain client: the sensor half of the REST contract (reference chronos_sensor.py:107-122).

Request  ``POST {brain}/api/generate`` with ``{"model": "llama3", "prompt": p, "stream": false, "format": "json"}``,
30 s timeout; the reply's ``response`` field is a string holding the verdict JSON.  Any failure (connect, timeout,
HTTP, JSON) becomes ``{"risk_score": 0, "verdict": "ERROR", "reason": str(e)}``.

:class:`BrainClient` is the blocking form (one chain in flight, as the reference).  :class:`AsyncBrainClient` fixes
quirk Q1: many chains in flight over a pooled connection, optional retries with jittered backoff,
and it can send the verdict JSON schema as ``format`` (Ollama structured outputs) instead of ``"json"``.
"""
from __future__ import annotations

import asyncio
import json
import random
import time
from dataclasses import dataclass
from typing import Any, Sequence

from .prompt import VERDICT_SCHEMA, build_prompt

DEFAULT_PORT = 11434
DEFAULT_MODEL = "llama3"
DEFAULT_TIMEOUT = 30.0


def brain_url(host: str, port: int = DEFAULT_PORT) -> str:
    if host.startswith("http://") or host.startswith("https://"):
        return host.rstrip("/") + ("" if host.rstrip("/").endswith("/api/generate") else "/api/generate")
    return f"http://{host}:{port}/api/generate"


def error_verdict(e: BaseException | str) -> dict:
    return {"risk_score": 0, "verdict": "ERROR", "reason": str(e)}


@dataclass
class ClientConfig:
    url: str = brain_url("127.0.0.1")
    model: str = DEFAULT_MODEL
    timeout: float = DEFAULT_TIMEOUT
    fmt: Any = "json"           # "json" (reference) or a JSON schema dict
    retries: int = 0            # reference: no retry
    backoff: float = 0.25
    options: dict | None = None  # forwarded Ollama options (num_predict, temperature, seed, ...)


def _body(cfg: ClientConfig, prompt: str) -> dict:
    body = {"model": cfg.model, "prompt": prompt, "stream": False, "format": cfg.fmt}
    if cfg.options:
        body["options"] = cfg.options
    return body


class BrainClient:
    def __init__(self, cfg: ClientConfig | None = None):
        import requests

        self.cfg = cfg or ClientConfig()
        self._session = requests.Session()

    def analyze(self, history: Sequence[str]) -> dict:
        prompt = build_prompt(history)
        last: BaseException | None = None
        for attempt in range(self.cfg.retries + 1):
            try:
                resp = self._session.post(self.cfg.url, json=_body(self.cfg, prompt), timeout=self.cfg.timeout)
                return json.loads(resp.json()["response"])
            except Exception as e:  # noqa: BLE001 — the contract maps every failure to an ERROR verdict
                last = e
                if attempt < self.cfg.retries:
                    time.sleep(self.cfg.backoff * (2 ** attempt) * (0.5 + random.random()))
        return error_verdict(last)


class AsyncBrainClient:
    """Pooled asyncio client (aiohttp).  ``max_inflight`` bounds concurrent requests per sensor."""

    def __init__(self, cfg: ClientConfig | None = None, max_inflight: int = 1024):
        self.cfg = cfg or ClientConfig()
        self._sem = asyncio.Semaphore(max_inflight)
        self._session = None
        self._max = max_inflight

    async def _sess(self):
        import aiohttp

        if self._session is None:
            conn = aiohttp.TCPConnector(limit=self._max, ttl_dns_cache=300)
            self._session = aiohttp.ClientSession(connector=conn)
        return self._session

    async def analyze(self, history: Sequence[str]) -> dict:
        import aiohttp

        prompt = build_prompt(history)
        sess = await self._sess()
        last: BaseException | None = None
        async with self._sem:
            for attempt in range(self.cfg.retries + 1):
                try:
                    tmo = aiohttp.ClientTimeout(total=self.cfg.timeout)
                    async with sess.post(self.cfg.url, json=_body(self.cfg, prompt), timeout=tmo) as resp:
                        data = await resp.json(content_type=None)
                    return json.loads(data["response"])
                except Exception as e:  # noqa: BLE001
                    last = e
                    if attempt < self.cfg.retries:
                        await asyncio.sleep(self.cfg.backoff * (2 ** attempt) * (0.5 + random.random()))
        return error_verdict(last)

    async def close(self):
        if self._session is not None:
            await self._session.close()
            self._session = None


def schema_format() -> dict:
    return dict(VERDICT_SCHEMA)

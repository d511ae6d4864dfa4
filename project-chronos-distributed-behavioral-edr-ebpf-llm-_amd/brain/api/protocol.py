"""Ollama REST protocol pieces.

The sensor's request (reference chronos_sensor.py:117-119):
    POST /api/generate {"model": "llama3", "prompt": ..., "stream": false, "format": "json"}
and it reads ``json.loads(resp.json()["response"])`` (:120).  Ollama's other generate fields (system, raw, options,
stream=true NDJSON, timing fields in ns) and /api/chat are served too so any Ollama client can talk to the Brain.
"""
from __future__ import annotations

import time
from dataclasses import dataclass
from typing import Any, Optional

OLLAMA_VERSION = "0.5.7-chronos"


class BadRequest(ValueError):
    pass


@dataclass
class GenerateParams:
    model: str = "llama3"
    prompt: str = ""
    messages: Optional[list] = None
    system: Optional[str] = None
    raw: bool = False
    stream: bool = True
    format: Any = None
    num_predict: int = 0
    temperature: float = 0.0
    seed: int = 0
    top_k: int = 0
    top_p: float = 1.0

    @classmethod
    def parse(cls, body: dict, chat: bool = False, default_temperature: float = 0.0) -> "GenerateParams":
        if not isinstance(body, dict):
            raise BadRequest("request body must be a JSON object")
        opts = body.get("options") or {}
        if not isinstance(opts, dict):
            raise BadRequest("options must be an object")
        fmt = body.get("format")
        if fmt not in (None, "", "json") and not isinstance(fmt, dict):
            raise BadRequest(f"invalid format {fmt!r}: use \"json\" or a JSON schema object")
        p = cls(
            model=str(body.get("model", "llama3")),
            prompt=str(body.get("prompt", "")),
            system=body.get("system"),
            raw=bool(body.get("raw", False)),
            stream=bool(body.get("stream", True)),  # Ollama's default is streaming
            format=fmt or None,
            num_predict=int(opts.get("num_predict", body.get("num_predict", 0)) or 0),
            temperature=float(opts.get("temperature", default_temperature)),
            seed=int(opts.get("seed", 0) or 0),
        )
        if p.temperature > 0:  # Ollama's sampler defaults apply whenever it samples (top_k 40, top_p 0.9)
            p.top_k = int(opts.get("top_k", 40) or 0)
            p.top_p = float(opts.get("top_p", 0.9))
        if chat:
            msgs = body.get("messages")
            if not isinstance(msgs, list) or not msgs:
                raise BadRequest("chat requires a non-empty messages list")
            for m in msgs:
                if not isinstance(m, dict) or "role" not in m:
                    raise BadRequest("each message needs a role and content")
            p.messages = msgs
        return p


def chat_prompt_ids(tok, messages: list) -> list:
    """Llama-3 multi-turn chat template."""
    from ..tokenizer import END_HEADER_ID, START_HEADER_ID

    ids = [tok.bos_id]
    for m in messages:
        ids += [START_HEADER_ID] + tok.encode(str(m["role"])) + [END_HEADER_ID]
        ids += tok.encode("\n\n" + str(m.get("content", ""))) + [tok.eot_id]
    ids += [START_HEADER_ID] + tok.encode("assistant") + [END_HEADER_ID] + tok.encode("\n\n")
    return ids


def _ns(s: float) -> int:
    return int(max(0.0, s) * 1e9)


def now_iso() -> str:
    t = time.time()
    return time.strftime("%Y-%m-%dT%H:%M:%S", time.gmtime(t)) + f".{int((t % 1) * 1e6):06d}Z"


def final_fields(req, load_duration: float = 0.0) -> dict:
    first = req.t_first or req.t_done
    return {
        "done": True,
        "done_reason": req.done_reason if req.done_reason != "error" else "stop",
        "total_duration": _ns(req.t_done - req.t_submit),
        "load_duration": _ns(load_duration),
        "prompt_eval_count": len(req.prompt_ids),
        "prompt_eval_duration": _ns(first - (req.t_admit or req.t_submit)),
        "eval_count": len(req.out_ids),
        "eval_duration": _ns(req.t_done - first),
    }


def generate_response(model: str, req) -> dict:
    d = {"model": model, "created_at": now_iso(), "response": req.text}
    d.update(final_fields(req))
    d["context"] = []
    return d


def chat_response(model: str, req) -> dict:
    d = {"model": model, "created_at": now_iso(), "message": {"role": "assistant", "content": req.text}}
    d.update(final_fields(req))
    return d

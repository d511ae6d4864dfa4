"""Ollama REST protocol pieces.

The sensor's request (reference chronos_sensor.py:117-119):
    POST /api/generate {"model": "llama3", "prompt": ..., "stream": false, "format": "json"}
and it reads ``json.loads(resp.json()["response"])`` (:120).  Ollama's other generate fields (system, raw, options,
stream=true NDJSON, timing fields in ns) and /api/chat are served too so any Ollama client can talk to the Brain:

* ``options.stop`` (string or list): generation ends at the first stop string, which is not part of the response;
* ``options.num_ctx``: the request's context window (prompt + generation), clamped to the engine's max_model_len — a
  prompt that does not fit is a 400, ``num_predict`` is clamped to what is left;
* ``context`` (request) continues from a previous reply's ``context`` (returned: prompt + generated token ids);
* ``keep_alive`` is accepted; the weights stay resident regardless (warm at start-up, quirk X8);
* ``options.repeat_penalty`` / ``frequency_penalty`` / ``presence_penalty`` are accepted and not applied (the
  verdict sampler is grammar-constrained greedy; a penalty != 1 / 0 is reported in the reply's ``ignored_options``).
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
    stop: tuple = ()
    num_ctx: int = 0
    context: Optional[list] = None
    keep_alive: Any = None
    ignored: tuple = ()

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
        stop = opts.get("stop", body.get("stop"))
        if stop is not None:
            stop = [stop] if isinstance(stop, str) else stop
            if not isinstance(stop, list) or not all(isinstance(x, str) for x in stop):
                raise BadRequest("options.stop must be a string or a list of strings")
            p.stop = tuple(x for x in stop if x)
        p.num_ctx = int(opts.get("num_ctx", 0) or 0)
        if p.num_ctx < 0:
            raise BadRequest("options.num_ctx must be positive")
        ctx = body.get("context")
        if ctx is not None:
            if not isinstance(ctx, list) or not all(isinstance(t, int) and t >= 0 for t in ctx):
                raise BadRequest("context must be a list of token ids")
            p.context = ctx
        p.keep_alive = body.get("keep_alive")
        p.ignored = tuple(k for k, neutral in (("repeat_penalty", 1.0), ("frequency_penalty", 0.0),
                                               ("presence_penalty", 0.0))
                          if k in opts and float(opts[k]) != neutral)
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


def generate_response(model: str, req, ignored: tuple = ()) -> dict:
    d = {"model": model, "created_at": now_iso(), "response": req.text}
    d.update(final_fields(req))
    # Ollama's continuation handle: the tokens of this exchange (template included); send it back as "context"
    d["context"] = [int(t) for t in list(req.prompt_ids) + list(req.out_ids)]
    if ignored:
        d["ignored_options"] = list(ignored)
    return d


def apply_stop(text: str, stop: tuple) -> tuple[str, bool]:
    """Cut ``text`` at the earliest occurrence of any stop string (Ollama: the stop string is not returned)."""
    cut = min((i for i in (text.find(s) for s in stop) if i >= 0), default=-1)
    return (text[:cut], True) if cut >= 0 else (text, False)


def stop_context_ids(tok, prompt_ids, out_ids, visible: str) -> list:
    """The continuation ``context`` of a reply cut at a stop string: the prompt, the generated tokens that lie wholly
    inside the text the client received, then the re-tokenised remainder of that text — never the stop string or
    what followed it (a continuation must not condition on text the client never saw)."""
    table = tok.token_bytes_list()
    vb = visible.encode("utf-8")
    pos, k = 0, 0
    for t in out_ids:
        b = table[t] if 0 <= t < len(table) else b""
        if not b or not vb.startswith(b, pos):
            break
        pos += len(b)
        k += 1
    rest = vb[pos:].decode("utf-8", errors="ignore")
    return [int(t) for t in list(prompt_ids) + list(out_ids[:k])] + ([int(t) for t in tok.encode(rest)] if rest else [])


def chat_response(model: str, req) -> dict:
    d = {"model": model, "created_at": now_iso(), "message": {"role": "assistant", "content": req.text}}
    d.update(final_fields(req))
    return d


class StopFilter:
    """Streaming form of ``apply_stop``: holds back the last (longest stop - 1) characters so a stop string split
    across chunks is still caught, and emits nothing after it."""

    def __init__(self, stop: tuple):
        self.stop = stop
        self.keep = max(len(x) for x in stop) - 1
        self.buf = ""
        self.hit = False

    def feed(self, text: str) -> str:
        if self.hit:
            return ""
        self.buf += text
        cut, hit = apply_stop(self.buf, self.stop)
        if hit:
            self.hit, self.buf = True, ""
            return cut
        if len(self.buf) > self.keep:
            out, self.buf = self.buf[:len(self.buf) - self.keep], self.buf[len(self.buf) - self.keep:]
            return out
        return ""

    def flush(self) -> str:
        out, self.buf = ("" if self.hit else self.buf), ""
        return out

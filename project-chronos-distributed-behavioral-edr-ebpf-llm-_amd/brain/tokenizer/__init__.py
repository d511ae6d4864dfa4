"""Tokenizers and the Llama-3 chat template for the Brain.

The reference's Brain (Ollama, ``llama3``) tokenised with Llama-3's 128,256-entry tiktoken BPE and wrapped the prompt
in the Llama-3 chat template before prefill.  No tokenizer assets exist offline, so:

* :class:`HFTokenizer` loads a real ``tokenizer.json`` (e.g. from a Llama-3 HF checkpoint dir) when one is given;
* :class:`ChronosBPE` is the default: a byte-level BPE trained offline on syscall-telemetry prompts + English/code text
  (``scripts/train_tokenizer.py``, asset ``assets/chronos_bpe.json``), with the Llama-3 special tokens at their real
  ids 128000-128255 and the model vocabulary kept at 128,256 so embedding / LM-head shapes match Llama-3 exactly.
  Its compression on CHRONOS prompts is close to Llama-3's (~3.5-4 chars/token), so benchmark sequence lengths are
  realistic.

Both expose ``encode``, ``decode``, ``token_bytes`` (raw bytes of every id, b"" for specials — what the grammar
compiler walks) and the special ids.
"""
from __future__ import annotations

import functools
import os
from typing import Sequence

VOCAB_SIZE = 128256
BOS_ID = 128000          # <|begin_of_text|>
EOT_TEXT_ID = 128001     # <|end_of_text|>
START_HEADER_ID = 128006  # <|start_header_id|>
END_HEADER_ID = 128007    # <|end_header_id|>
EOT_ID = 128009          # <|eot_id|>

_SPECIAL_NAMES = {
    128000: "<|begin_of_text|>",
    128001: "<|end_of_text|>",
    128002: "<|reserved_special_token_0|>",
    128003: "<|reserved_special_token_1|>",
    128004: "<|finetune_right_pad_id|>",
    128005: "<|reserved_special_token_2|>",
    128006: "<|start_header_id|>",
    128007: "<|end_header_id|>",
    128008: "<|eom_id|>",
    128009: "<|eot_id|>",
    128010: "<|python_tag|>",
}

ASSET = os.path.join(os.path.dirname(os.path.abspath(__file__)), "assets", "chronos_bpe.json")


def special_name(i: int) -> str:
    return _SPECIAL_NAMES.get(i, f"<|reserved_special_token_{i - 128000 - 3}|>")


@functools.lru_cache(maxsize=1)
def _byte_decoder() -> dict[str, int]:
    """Inverse of GPT-2's bytes_to_unicode (the ByteLevel pre-tokenizer's alphabet)."""
    bs = list(range(ord("!"), ord("~") + 1)) + list(range(ord("¡"), ord("¬") + 1)) + list(range(ord("®"), ord("ÿ") + 1))
    cs = bs[:]
    n = 0
    for b in range(256):
        if b not in bs:
            bs.append(b)
            cs.append(256 + n)
            n += 1
    return {chr(c): b for b, c in zip(bs, cs)}


class _Base:
    vocab_size = VOCAB_SIZE
    bos_id = BOS_ID
    eot_id = EOT_ID
    stop_ids: tuple[int, ...] = (EOT_ID, EOT_TEXT_ID)

    def encode(self, text: str) -> list[int]:
        raise NotImplementedError

    def decode(self, ids: Sequence[int]) -> str:
        tb = self.token_bytes_list()
        n = len(tb)
        return b"".join([tb[i] for i in ids if 0 <= i < n]).decode("utf-8", errors="replace")

    def token_bytes_list(self) -> list[bytes]:
        raise NotImplementedError

    def chat_ids(self, prompt: str, system: str | None = None, raw: bool = False) -> list[int]:
        """Llama-3 chat template (what Ollama applies to /api/generate prompts unless raw=true)."""
        if raw:
            return [self.bos_id] + self.encode(prompt)
        ids = [self.bos_id]
        if system:
            ids += [START_HEADER_ID] + self.encode("system") + [END_HEADER_ID] + self.encode("\n\n" + system) + [EOT_ID]
        ids += [START_HEADER_ID] + self.encode("user") + [END_HEADER_ID] + self.encode("\n\n" + prompt) + [EOT_ID]
        ids += [START_HEADER_ID] + self.encode("assistant") + [END_HEADER_ID] + self.encode("\n\n")
        return ids


class ChronosBPE(_Base):
    def __init__(self, path: str = ASSET):
        from tokenizers import Tokenizer

        if not os.path.exists(path):
            raise FileNotFoundError(f"tokenizer asset missing: {path} (run scripts/train_tokenizer.py)")
        self._tok = Tokenizer.from_file(path)
        self.n_bpe = self._tok.get_vocab_size()
        assert self.n_bpe < BOS_ID
        self._bytes: list[bytes] | None = None
        import regex

        # The ByteLevel pre-tokenizer splits text with the GPT-2 pattern and BPE never merges across pieces, so
        # caching each piece's ids is exact.  Telemetry pieces (paths, comms, template words) repeat constantly:
        # this halves the host-side tokenizer cost of a 1024-chain wave (tests/test_brain_cpu.py checks equality).
        self._pat = regex.compile(r"""'s|'t|'re|'ve|'m|'ll|'d| ?\p{L}+| ?\p{N}+| ?[^\s\p{L}\p{N}]+|\s+(?!\S)|\s+""")
        self._pieces: dict[str, list[int]] = {}

    def encode(self, text: str) -> list[int]:
        out: list[int] = []
        cache = self._pieces
        for piece in self._pat.findall(text):
            ids = cache.get(piece)
            if ids is None:
                ids = self._tok.encode(piece, add_special_tokens=False).ids
                if len(cache) < 1_000_000:
                    cache[piece] = ids
            out += ids
        return out

    def encode_uncached(self, text: str) -> list[int]:
        return self._tok.encode(text, add_special_tokens=False).ids

    def encode_batch(self, texts: Sequence[str]) -> list[list[int]]:
        return [e.ids for e in self._tok.encode_batch(list(texts), add_special_tokens=False)]

    def token_bytes_list(self) -> list[bytes]:
        if self._bytes is None:
            dec = _byte_decoder()
            vocab = self._tok.get_vocab()
            out = [b""] * VOCAB_SIZE
            for s, i in vocab.items():
                out[i] = bytes(dec[c] for c in s)
            self._bytes = out
        return self._bytes


class HFTokenizer(_Base):
    """A real ``tokenizer.json`` (e.g. Meta-Llama-3-8B-Instruct).  Special tokens come from the file itself."""

    def __init__(self, path: str):
        from tokenizers import Tokenizer

        if os.path.isdir(path):
            path = os.path.join(path, "tokenizer.json")
        self._tok = Tokenizer.from_file(path)
        self.vocab_size = max(VOCAB_SIZE, self._tok.get_vocab_size())
        self._bytes: list[bytes] | None = None
        v = self._tok.get_vocab()
        self.bos_id = v.get("<|begin_of_text|>", BOS_ID)
        self.eot_id = v.get("<|eot_id|>", EOT_ID)
        self.stop_ids = tuple(x for x in (v.get("<|eot_id|>"), v.get("<|end_of_text|>")) if x is not None)

    def encode(self, text: str) -> list[int]:
        return self._tok.encode(text, add_special_tokens=False).ids

    def encode_batch(self, texts: Sequence[str]) -> list[list[int]]:
        return [e.ids for e in self._tok.encode_batch(list(texts), add_special_tokens=False)]

    def token_bytes_list(self) -> list[bytes]:
        if self._bytes is None:
            dec = _byte_decoder()
            out = [b""] * self.vocab_size
            specials = {t.content for t in self._tok.get_added_tokens_decoder().values()}
            for s, i in self._tok.get_vocab().items():
                if s in specials:
                    continue
                try:
                    out[i] = bytes(dec[c] for c in s)
                except KeyError:  # non-byte-level vocab: fall back to UTF-8 of the piece
                    out[i] = s.replace("▁", " ").encode()
            self._bytes = out
        return self._bytes


def load_tokenizer(path: str | None = None) -> _Base:
    if path:
        cand = os.path.join(path, "tokenizer.json") if os.path.isdir(path) else path
        if os.path.exists(cand):
            return HFTokenizer(cand)
    return ChronosBPE()

"""Kill-chain prompt builder.

The prompt bytes are part of the sensor->Brain contract: they must equal the reference
f-string at chronos_sensor.py:109-114 for every history, including the leading newline, the 4-space indentation
and the trailing newline + 4 spaces, with the history rendered as Python ``str(list)``.
"""
from __future__ import annotations

from typing import Sequence

_HEAD = "\n    Analyze this sequence. Return JSON ONLY.\n    Sequence: "
_TAIL = (
    "\n    Context: 'curl' -> 'chmod' -> 'exec' is a Dropper."
    '\n    Format: {"risk_score": <0-10>, "verdict": "<SAFE/MALICIOUS>", "reason": "<Short Explanation>"}'
    "\n    "
)

# The verdict schema the prompt asks for; the Brain's schema-constrained decoder enforces exactly this shape.
VERDICT_SCHEMA = {
    "type": "object",
    "properties": {
        "risk_score": {"type": "integer", "minimum": 0, "maximum": 10},
        "verdict": {"type": "string", "enum": ["SAFE", "MALICIOUS"]},
        "reason": {"type": "string"},
    },
    "required": ["risk_score", "verdict", "reason"],
}


def build_prompt(history: Sequence[str]) -> str:
    return _HEAD + str(list(history)) + _TAIL


def prompt_prefix() -> str:
    """History-independent head of every prompt (shared by all chains: prefix-cache candidate)."""
    return _HEAD + "["

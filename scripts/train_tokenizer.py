"""Train the offline CHRONOS byte-level BPE (asset for chronos.brain.tokenizer.ChronosBPE).

Corpus (deterministic): CHRONOS kill-chain prompts built from synthetic fleet telemetry + the attack_chain.sh replay,
verdict-shaped JSON, and English/code text taken from the Python standard library's docstrings on this image.
Usage: python scripts/train_tokenizer.py [--vocab 32000]
"""
from __future__ import annotations

import argparse
import ast
import glob
import json
import os
import random
import sys
import sysconfig

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def corpus(seed: int = 0):
    from chronos.sensor.prompt import build_prompt
    from chronos.sensor.replay import synthetic_chains

    rng = random.Random(seed)
    for t in synthetic_chains(20000, seed=seed, native=False):
        yield build_prompt(t.history)
    words = ["curl", "chmod", "dropper", "download", "payload", "executable", "suspicious", "benign", "shell",
             "script", "network", "file", "write", "permission", "binary", "malware", "process", "sequence",
             "pattern", "activity", "consistent", "with", "normal", "system", "user", "the", "a", "of", "and", "to"]
    for _ in range(20000):
        reason = " ".join(rng.choice(words) for _ in range(rng.randint(3, 14))).capitalize() + "."
        yield json.dumps({"risk_score": rng.randint(0, 10), "verdict": rng.choice(["SAFE", "MALICIOUS"]),
                          "reason": reason})
    stdlib = sysconfig.get_paths()["stdlib"]
    for path in sorted(glob.glob(os.path.join(stdlib, "*.py")))[:400]:
        try:
            src = open(path, encoding="utf-8").read()
        except Exception:
            continue
        yield src
        try:
            tree = ast.parse(src)
        except SyntaxError:
            continue
        for node in ast.walk(tree):
            if isinstance(node, (ast.FunctionDef, ast.ClassDef, ast.Module)):
                d = ast.get_docstring(node)
                if d:
                    yield d


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--vocab", type=int, default=32000)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    from tokenizers import Tokenizer, decoders, models, pre_tokenizers, trainers

    from chronos.brain.tokenizer import ASSET

    tok = Tokenizer(models.BPE())
    tok.pre_tokenizer = pre_tokenizers.ByteLevel(add_prefix_space=False, use_regex=True)
    tok.decoder = decoders.ByteLevel()
    trainer = trainers.BpeTrainer(vocab_size=a.vocab, min_frequency=2, show_progress=False,
                                  initial_alphabet=pre_tokenizers.ByteLevel.alphabet())
    tok.train_from_iterator(corpus(), trainer=trainer)
    out = a.out or ASSET
    os.makedirs(os.path.dirname(out), exist_ok=True)
    tok.save(out)
    print(f"saved {out}: vocab {tok.get_vocab_size()}")


if __name__ == "__main__":
    main()

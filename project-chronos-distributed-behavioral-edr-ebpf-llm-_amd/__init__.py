"""CHRONOS-MI355X: a behavioral EDR analysis node with an MI355X-native Llama-3 "Brain".

Layout:
  sensor/    N0-N2  eBPF program + shared filter header, BCC loader, replay/synthetic sources, chain tracker,
                    byte-exact prompt builder, Brain client, verdict renderer     (reference: chronos_sensor.py)
  brain/     N3-N4  Ollama-compatible REST API, continuous-batching engine, paged-KV block manager,
                    tokenizer + chat template, JSON / verdict-schema constrained decoding
  models/    N5     Llama-3 / 3.1 (8B, 70B, 128k) definition, checkpoint loaders, random init
  ops/       N7     gfx950 HIP kernels (csrc/kernels) + their pure-torch fp32 oracles
  parallel/  N6     process groups (RCCL over xGMI / gloo), tensor-parallel layers, custom all-reduce, DP router
  utils/            metrics, timing, logging helpers

Import it as ``chronos`` (the repo-root alias package).
"""

__version__ = "0.1.0"

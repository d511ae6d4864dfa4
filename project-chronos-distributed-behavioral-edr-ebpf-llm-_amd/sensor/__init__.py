"""CHRONOS sensor: eBPF program, event sources, chain tracker, prompt, Brain client, renderer."""

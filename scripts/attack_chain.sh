#!/bin/bash
# MITRE ATT&CK T1105 (ingress tool transfer) dropper simulation — the CHRONOS end-to-end scenario.
# Same three observable steps as the reference scenario (attack_chain.sh:1-16): a download redirected into
# /tmp/malware.bin, a permission change, and a read of the payload standing in for its execution.
# Usage: ./scripts/attack_chain.sh [URL]   (no network? the download step simply writes an empty file)
set -u
URL="${1:-https://www.google.com}"
PAYLOAD=/tmp/malware.bin
echo "--- Initiating Dropper Simulation (MITRE T1105) ---"
curl -s "$URL" > "$PAYLOAD"          # network event: download
chmod +x "$PAYLOAD"                  # file event: make it executable
cat "$PAYLOAD" > /dev/null           # execution event (simulated)
echo "--- Kill Chain Complete ---"

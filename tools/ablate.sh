#!/bin/bash
# Diagnostic: dense-round gossip scatter time with parts of the work removed (results wrong).
cd "$(dirname "$0")/.."
for a in 0 1 2 4 7; do
  P2PG_GOSSIP_PUSH=store P2PG_ABLATE=$a timeout -k 10 200 python3 tools/round_profile.py c4 1 > gpurun_out/ablate_$a.json 2>/dev/null || echo "ablate $a failed"
done

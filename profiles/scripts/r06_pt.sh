#!/bin/bash
# Round 6, final kernels: the pilot sample beside the long-row wide pass (C2 / C3: 1M rows, 512
# tiles by default) at 256 and 128 tiles.
set -o pipefail
AB="c2|--steps 200;c2p256|--steps 200 --pilot-tiles 256;c2p128|--steps 200 --pilot-tiles 128;c3|--config c3 --steps 100;c3p256|--config c3 --steps 100 --pilot-tiles 256;c3p128|--config c3 --steps 100 --pilot-tiles 128" \
  ROUNDS=2 T=240 bash profiles/scripts/r06_ab.sh

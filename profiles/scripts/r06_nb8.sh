#!/bin/bash
# Round 6: the 8-wave finish (D > 1024: C3) with 3 / 4 long rows per wave per batch
# (VDB_FIN_NB8; default 2) -- same-box A/B at C3, C2 as the control.
set -o pipefail
L=mlx-vector-db_amd/lib/libvdb_amd
AB="c3|--config c3 --steps 100;c3n3|VDB_LIB=${L}_nb3.so --config c3 --steps 100;c3n4|VDB_LIB=${L}_nb4.so --config c3 --steps 100;c2|--steps 200;c2n4|VDB_LIB=${L}_nb4.so --steps 200" \
  ROUNDS=2 T=240 bash profiles/scripts/r06_ab.sh

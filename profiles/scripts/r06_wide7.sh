#!/bin/bash
# Round 6: wide pass -- H products first (tile tests under the L MFMAs), with / without a stagger.
set -o pipefail
L=mlx-vector-db_amd/lib
export AB="wide|--config c4;hf|VDB_LIB=$L/libvdb_amd_hf.so --config c4;hfst8|VDB_LIB=$L/libvdb_amd_hfst8.so --config c4"
ROUNDS=2 T=200 bash profiles/scripts/r06_ab.sh

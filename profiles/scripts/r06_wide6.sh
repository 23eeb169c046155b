#!/bin/bash
# Round 6: wide pass -- the next tile's LDS reads issued after this tile's first MFMA group.
set -o pipefail
L=mlx-vector-db_amd/lib
export AB="wide|--config c4;pf|VDB_LIB=$L/libvdb_amd_pf.so --config c4;pfkl|VDB_LIB=$L/libvdb_amd_pfkl.so --config c4 --no-fallback;wkl|VDB_LIB=$L/libvdb_amd_wkl.so --config c4 --no-fallback"
ROUNDS=2 T=200 bash profiles/scripts/r06_ab.sh

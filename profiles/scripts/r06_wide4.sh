#!/bin/bash
# Round 6: wide pass -- LDS prefetch of the next tile, stagger of each SIMD's second wave.
set -o pipefail
L=mlx-vector-db_amd/lib
export AB="wide|--config c4;pf|VDB_LIB=$L/libvdb_amd_pf.so --config c4;st4|VDB_LIB=$L/libvdb_amd_st4.so --config c4;st8|VDB_LIB=$L/libvdb_amd_st8.so --config c4;pfst8|VDB_LIB=$L/libvdb_amd_pfst8.so --config c4"
ROUNDS=2 T=200 bash profiles/scripts/r06_ab.sh

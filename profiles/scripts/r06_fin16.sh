#!/bin/bash
# Round 6: the finish's int8 refinement with 16 rows per wave in flight (VDB_FIN_NBR=16, one HBM
# round for KP <= 256) against the default 4: phase stamps, then bench A/B (3 streams; p50 = one
# batch at a time).
set -o pipefail
O=gpurun_out/r06_fin16; mkdir -p $O
export VDB_LIB=mlx-vector-db_amd/lib/libvdb_amd_st16.so
FIN_ROWS=1250000 timeout -k 10 120 python -u profiles/scripts/fin_stamp.py c6 auto > $O/fin_c6shard.txt 2>&1 || { tail -20 $O/fin_c6shard.txt; exit 1; }
timeout -k 10 120 python -u profiles/scripts/fin_stamp.py c2 auto > $O/fin_c2.txt 2>&1 || { tail -20 $O/fin_c2.txt; exit 1; }
timeout -k 10 120 python -u profiles/scripts/fin_stamp.py c3 auto > $O/fin_c3.txt 2>&1 || { tail -20 $O/fin_c3.txt; exit 1; }
unset VDB_LIB
grep -v amdgpu $O/fin_*.txt
L=mlx-vector-db_amd/lib/libvdb_amd_r16.so
AB="c2|--config c2 --steps 200;c2r16|VDB_LIB=$L --config c2 --steps 200;c3|--config c3 --steps 100;c3r16|VDB_LIB=$L --config c3 --steps 100;sh|--config c6 --rows 1250000 --steps 400;shr16|VDB_LIB=$L --config c6 --rows 1250000 --steps 400" \
  ROUNDS=2 T=200 bash profiles/scripts/r06_ab.sh

#!/bin/bash
# Round 6: rows of > 1024 dims (C3) finished by a 16-wave form compiled for long rows alone (one
# row per wave per batch, 126 VGPRs, no spills; VDB_FIN_W16L=1) against the 8-wave form: the
# parity tests on the variant, then same-box A/B at C3 (B = 256 and 16).
set -o pipefail
O=gpurun_out/r06_w16l; mkdir -p $O
L=mlx-vector-db_amd/lib/libvdb_amd_w16l.so
VDB_LIB=$L timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_wide.py -x -q \
  --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
AB="c3|--config c3 --steps 100;c3l|VDB_LIB=$L --config c3 --steps 100;c3b16|--config c3 --batch 16 --steps 100;c3b16l|VDB_LIB=$L --config c3 --batch 16 --steps 100" \
  ROUNDS=2 T=240 bash profiles/scripts/r06_ab.sh

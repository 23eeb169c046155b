#!/bin/bash
# Round 6: the wide pass with a one-tile-ahead operand prefetch (ping-pong register sets,
# VDB_W8_PP=1; + raised priority for the H MFMAs, VDB_W8_PRIO=1): parity of the wide tests on the
# prefetch build, then A/B against the main library and the refactored default (w0) on C4 and
# the c4 shard shape.
set -o pipefail
O=gpurun_out/r06_wpp; mkdir -p $O
VDB_LIB=mlx-vector-db_amd/lib/libvdb_amd_wppp.so timeout -k 10 300 python -u -m pytest tests/test_gpu_wide.py -x -q \
  --timeout 120 --timeout-method thread > $O/pytest_wppp.txt 2>&1 || { tail -30 $O/pytest_wppp.txt; exit 1; }
tail -1 $O/pytest_wppp.txt
L=mlx-vector-db_amd/lib/libvdb_amd
AB="c4|--config c4 --steps 100;c4w0|VDB_LIB=${L}_w0.so --config c4 --steps 100;c4pp|VDB_LIB=${L}_wpp.so --config c4 --steps 100;c4ppp|VDB_LIB=${L}_wppp.so --config c4 --steps 100;s4|--config c4 --rows 1250000 --steps 200;s4pp|VDB_LIB=${L}_wpp.so --config c4 --rows 1250000 --steps 200;s4ppp|VDB_LIB=${L}_wppp.so --config c4 --rows 1250000 --steps 200" \
  ROUNDS=2 T=240 bash profiles/scripts/r06_ab.sh

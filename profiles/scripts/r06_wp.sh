#!/bin/bash
# Round 6: the wide pass with its H MFMAs at raised wave priority (VDB_W8_PRIO=1) against the
# default, C4 and the c4 shard shape (1.25M x 128, B = 512).
set -o pipefail
L=mlx-vector-db_amd/lib/libvdb_amd_wp.so
AB="c4|--config c4 --steps 100;c4wp|VDB_LIB=$L --config c4 --steps 100;s4|--config c4 --rows 1250000 --steps 200;s4wp|VDB_LIB=$L --config c4 --rows 1250000 --steps 200" \
  ROUNDS=2 T=240 bash profiles/scripts/r06_ab.sh

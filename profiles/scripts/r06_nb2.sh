#!/bin/bash
# Round 6: C3's finish with two 1536-dim rows per wave per exact-key batch (nb2) now that it never
# runs beside the scan.
set -o pipefail
L=mlx-vector-db_amd/lib/libvdb_amd_nb2.so
AB="c3|--config c3 --steps 100;c3n|VDB_LIB=$L --config c3 --steps 100" ROUNDS=3 T=200 bash profiles/scripts/r06_ab.sh

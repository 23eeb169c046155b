#!/bin/bash
# Round 6 diagnostic: is the wide pass's K-loop bound by its LDS bytes?  Builds with one LDS read of
# the L2 start values per tile instead of four (wnr; results garbage, run without fallback), with
# and without the epilogue (KLOOP_ONLY: wkl / wnrkl), against the main library, C4.
set -o pipefail
L=mlx-vector-db_amd/lib/libvdb_amd
AB="c4|--config c4 --steps 100;wnr|VDB_LIB=${L}_wnr.so --config c4 --steps 100 --no-fallback;wkl|VDB_LIB=${L}_wkl.so --config c4 --steps 100 --no-fallback;wnrkl|VDB_LIB=${L}_wnrkl.so --config c4 --steps 100 --no-fallback" \
  ROUNDS=2 T=240 bash profiles/scripts/r06_ab.sh

#!/bin/bash
# Round 6: where the wide pass's epilogue goes -- no insertions, pilot bound tightness.
set -o pipefail
export AB="wide|--config c4;wni|VDB_LIB=mlx-vector-db_amd/lib/libvdb_amd_wni.so --config c4 --no-fallback;pr3|--config c4 --pilot-rank 3 --no-fallback;pr8|--config c4 --pilot-rank 8 --no-fallback;pt16|--config c4 --pilot-tiles 16384;ck0|--config c4 --scan-checksum 0"
ROUNDS=2 T=200 bash profiles/scripts/r06_ab.sh

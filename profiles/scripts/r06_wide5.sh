#!/bin/bash
set -o pipefail
TAG=r06w_c4 bash profiles/scripts/r06_pmc.sh --config c4 && TAG=r06wkl_c4 LIB=mlx-vector-db_amd/lib/libvdb_amd_wkl.so bash profiles/scripts/r06_pmc.sh --config c4 --no-fallback

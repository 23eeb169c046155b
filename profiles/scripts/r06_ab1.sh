export AB="base|--config c4;kl|VDB_LIB=mlx-vector-db_amd/lib/libvdb_amd_kl.so --config c4 --no-fallback;ck0|--config c4 --scan-checksum 0;pr3|--config c4 --pilot-rank 3 --no-fallback;pt16k|--config c4 --pilot-tiles 16384"
ROUNDS=2 T=200 bash profiles/scripts/r06_ab.sh

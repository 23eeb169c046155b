"""Mirror of the reference ``performance`` package (performance/mlx_optimized.py,
performance/hnsw_index.py) on the gfx950 core."""

"""Shared pytest setup.

* ``-m "not gpu"`` (CPU, runs anywhere): oracle vs golden fixtures and the
  reference's known-answer pins, host logic of the store, the C-ABI library
  loading and exporting every symbol of include/vdb.h, multi-rank merge logic
  over gloo.
* ``-m gpu`` (an MI355X): parity of the HIP path, through the C-ABI, against
  the oracle.
"""
import os
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
PKG = os.path.join(ROOT, "mlx-vector-db_amd")
for p in (PKG, ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) and the built HIP library")
    config.addinivalue_line("markers", "slow: full-size (BASELINE.json config) case")

"""pytest configuration: the `gpu` marker and import paths.

`-m "not gpu"` runs on any host (oracle vs golden fixtures, host logic, the
C-ABI library loading and exporting every symbol of include/pmm.h).  `-m gpu`
needs a gfx950 device and runs the parity tests through the C ABI.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "polars-matmul_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) device")

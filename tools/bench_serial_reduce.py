"""bench.py with the weight-gradient split-K reductions in stream order on the main stream (ops.Workspace overlap off):
the A/B arm for the side-stream reductions.   python tools/bench_serial_reduce.py <bench.py arguments>"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import climsr_amd  # noqa: E402,F401
from climsr_amd import ops  # noqa: E402

_init = ops.Workspace.__init__


def _serial_init(self, overlap=False):
    _init(self, overlap=False)


ops.Workspace.__init__ = _serial_init
import bench  # noqa: E402

sys.exit(bench.main(sys.argv[1:]))

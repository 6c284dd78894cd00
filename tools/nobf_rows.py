"""A/B helper: run bench.py with the amp D = 64 projections on the fp32-operand GEMM kernels (the pre-rowgemm_bf
routing), e.g. `python tools/nobf_rows.py --config cfg4 --steps 6 --warmup 3 --no-cpu-baseline`."""
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "toss-next-ctr-prediction_amd"))
from tossctr import _lib  # noqa: E402

_query = _lib.query
_lib.query = lambda name, *a: 0 if name == "ctr_rowgemm_bf_supported" else _query(name, *a)
sys.argv = [os.path.join(ROOT, "bench.py")] + sys.argv[1:]
runpy.run_path(sys.argv[0], run_name="__main__")

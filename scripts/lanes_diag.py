"""Is the lane path bitwise reproducible? Runs the test_gpu_federation config twice per lane count."""
import sys, os, tempfile
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import bcfl  # noqa
from test_gpu_federation import _run

routes = sys.argv[1:] or [""]
for route in routes:
    os.environ["BCFL_TORCH_OPS"] = route
    outs = {}
    for lanes in (1, 3):
        for rep in range(2):
            outs[(lanes, rep)] = _run(tempfile.mkdtemp(), lanes, False)[0]
    ref = outs[(1, 0)]
    print(f"[{route}]", {k: float((v - ref).abs().max()) for k, v in outs.items()}, flush=True)

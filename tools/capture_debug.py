import os, sys, traceback
os.environ["DL4J_AMD_CAPTURE_DEBUG"]="1"
sys.path.insert(0, os.getcwd())
import torch
from deeplearning4j_amd.ops import native
import deeplearning4j_amd.nn.hipgraph as HG
# trace every torch op during capture via a dispatch mode to find the first op after which capture is invalid
from torch.utils._python_dispatch import TorchDispatchMode
class Probe(TorchDispatchMode):
    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        out = func(*args, **(kwargs or {}))
        if native.capture_status() == 2:
            raise RuntimeError(f"capture invalidated after torch op {func}")
        return out
orig_body = HG.CapturedTrainingStep._body
def body(self):
    with Probe():
        return orig_body(self)
HG.CapturedTrainingStep._body = body
sys.argv = ["bench.py", "--steps", "3", "--warmup", "2", "--graph", "1", "--batch", "32"]
import runpy
try:
    runpy.run_path("bench.py", run_name="__main__")
except Exception:
    traceback.print_exc()

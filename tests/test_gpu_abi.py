"""The C-only ABI driver on the GPU (tests/native/abi_driver.c): GEMM (bf16 LDS-DMA MFMA kernel and exact-fp32
kernel), 3x3 convolution, the fused updater and an RCCL all-reduce, each through csrc/include/dl4j_amd.h alone,
checked against host references inside the driver."""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu


def test_abi_driver_on_gpu():
    from deeplearning4j_amd.ops.build import ABI_DRIVER
    assert os.path.exists(ABI_DRIVER), "run the build first (ops/build.py build_abi_driver)"
    r = subprocess.run([ABI_DRIVER], capture_output=True, text=True, timeout=110)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ABI OK" in r.stdout and "matmul bf16" in r.stdout and "RCCL" in r.stdout

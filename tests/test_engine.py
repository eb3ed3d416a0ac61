"""Native engine (csrc/engine.hip) on the CPU host: the library loads, the op registry resolves every
listed kernel entry point in the library itself, and device queries degrade cleanly without a GPU."""
import torch

from deeplearning4j_amd import runtime as rt


def test_op_registry_resolves_entry_points():
    ops = rt.ops()
    assert len(ops) >= 30
    names = [o[0] for o in ops]
    assert len(set(names)) == len(names)
    for name, sig, what, has_fn in ops:
        assert name.startswith("dl4j_") and sig.startswith("int(") and what
        assert has_fn, f"{name} is not exported by the kernel library"
    assert "dl4j_gemm" in names and "dl4j_bn_bwd" in names and "dl4j_lstm_fwd_coop" in names


def test_device_queries_without_gpu():
    if torch.cuda.is_available():
        assert rt.device_count() >= 1
    else:
        assert rt.device_count() == 0
        assert rt.device_buffer(1024, "cpu") is None


def test_workspace_buffer_on_cpu_is_torch():
    from deeplearning4j_amd.memory.workspace import _device_buffer
    b = _device_buffer(4096, "cpu")
    assert b.dtype == torch.uint8 and b.numel() == 4096 and b.device.type == "cpu"

"""Native engine on the MI355X (csrc/engine.hip): device properties, the stream-ordered caching allocator (reuse,
splitting / coalescing, cross-stream deferral, DLPack tensors, empty_cache), native streams / events, and HIP-graph
capture with a private allocation pool."""
import pytest
import torch

from deeplearning4j_amd import runtime as rt

pytestmark = pytest.mark.gpu


def test_device_props():
    assert rt.device_count() >= 1
    p = rt.device_props(0)
    assert p["arch"].startswith("gfx950"), p
    assert p["cus"] >= 200 and p["warp"] == 64 and p["total_mem"] > 100 * 2 ** 30
    free, total = rt.mem_info(0)
    assert 0 < free <= total


def test_allocator_reuse_split_coalesce():
    a = rt.Allocator(0)
    s0 = a.stats()
    p1 = a.malloc(3 << 20)               # large: 4 MB block carved from a >= 64 MB segment
    p2 = a.malloc(5 << 20)
    st = a.stats()
    assert st["allocated"] - s0["allocated"] == (4 << 20) + (6 << 20)
    a.free(p2)
    a.free(p1)
    # both return to the pool and coalesce with the rest of their segment: a 10 MB request is served from the cache
    seg = a.stats()["segments"]
    hits = a.stats()["cache_hits"]
    p3 = a.malloc(9 << 20)
    assert a.stats()["segments"] == seg and a.stats()["cache_hits"] == hits + 1
    a.free(p3)
    q = [a.malloc(1000) for _ in range(8)]    # small: 1024-byte blocks of one 2 MB segment
    assert len(set(q)) == 8 and max(q) - min(q) < (2 << 20)
    for x in q:
        a.free(x)


def test_allocator_cross_stream_deferral():
    a = rt.Allocator(0)
    s1 = rt.Stream(0)
    t = a.empty((1 << 20,), torch.float32)
    ts = s1.torch_stream()
    with torch.cuda.stream(ts):
        torch.cuda._sleep(20_000_000)            # keep the side stream busy
        t.add_(1.0)
    a.record_stream(t.data_ptr(), s1)
    ptr = t.data_ptr()
    del t                                        # freed while the side stream still uses it
    u = a.empty((1 << 20,), torch.float32)
    assert u.data_ptr() != ptr                   # not handed out before the side stream's event completes
    s1.synchronize()
    del u


def test_dlpack_tensor_lifecycle():
    a = rt.Allocator(0)
    before = a.stats()["allocated"]
    x = a.empty((256, 1024), torch.bfloat16)
    assert x.is_cuda and x.dtype == torch.bfloat16 and x.shape == (256, 1024) and x.is_contiguous()
    x.copy_(torch.randn(256, 1024, device="cuda").to(torch.bfloat16))
    y = (x.float() * 2).sum()
    assert torch.isfinite(y)
    assert a.stats()["allocated"] > before
    del x
    torch.cuda.synchronize()
    assert a.stats()["allocated"] == before
    b = rt.device_buffer(12345, "cuda:0")
    assert b.numel() == 12345 and b.dtype == torch.uint8


def test_streams_events_timing():
    s = rt.Stream(0, high_priority=True)
    e0, e1 = rt.Event(), rt.Event()
    e0.record(s)
    with torch.cuda.stream(s.torch_stream()):
        torch.cuda._sleep(5_000_000)
    e1.record(s)
    e1.synchronize()
    assert e1.query() and s.query()
    assert e0.elapsed_ms(e1) > 0.1


def test_graph_capture_private_pool_and_replay():
    s = rt.Stream(0)
    a = rt.allocator(0)
    ts = s.torch_stream()
    x = torch.ones(1 << 16, device="cuda")
    # warm the stream: a free block of this stream the capture can take into its private pool
    w = a.empty((1 << 16,), torch.float32, stream=s)
    del w
    torch.cuda.synchronize()
    g = rt.Graph(s)
    with torch.cuda.stream(ts):
        g.capture_begin(rt.Graph.CAPTURE_RELAXED)
        tmp = a.empty((1 << 16,), torch.float32, stream=s)   # served from the capture pool, no hipMalloc
        tmp.copy_(x)
        x.add_(tmp)
        g.capture_end()
    assert g.num_nodes() >= 2
    for _ in range(3):
        g.replay()
    s.synchronize()
    assert float(x[0]) == 8.0                    # 1 -> 2 -> 4 -> 8
    del tmp
    g.destroy()
    assert a.empty_cache() >= 0

"""``mmul`` — the framework's matrix multiply, on the in-tree MFMA kernels of ``csrc/gemm.hip``.

    C = act(alpha * A @ B + bias + beta * C)          A [.., M, K], B [.., K, N]  (optional 3-D batch)

Reference call sites this serves: nn/layers/BaseLayer.java:86,97,334-336 (preOutput, backprop dW / eps),
BaseOutputLayer.java:151,178, recurrent/LSTMHelpers.java:206,212,522,616-676, SameDiff ``mmul``.

* Transposes are free: a transposed torch view only changes the operand-layout flag handed to the kernel
  (K- vs M/N-contiguous). A column-major destination (e.g. a DL4J 'f'-order weight-gradient view) is filled as
  C^T = B^T A^T by swapping the operands.
* bf16 / fp16 operands with 16-byte-addressable layouts run the LDS-DMA MFMA kernel (fp32 accumulation, split-K
  with a deterministic reduce when the tile grid alone cannot fill 256 CUs); fp32 operands and odd layouts run the
  exact-fp32 MFMA kernel. fp64 (gradient checks) and CPU tensors use torch — on a GPU tensor that is counted as a
  helper fallback (``ops.fallback``).
* Everything launches on torch's current stream (HIP-graph capturable); split-K slabs come from torch's caching
  allocator.
"""
import ctypes
import os

import torch

from . import fallback, tunedb
from .dispatch import use_native

_DT = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2}
ACT = {None: 0, "identity": 0, "relu": 1, "tanh": 2, "sigmoid": 3, "gelu": 4,
       "dgelu": 5}                                      # dgelu: out *= gelu'(z), z READ from the ``z`` buffer
_c = ctypes
_sig_done = [False]
_env = os.environ.get("DL4J_AMD_GEMM_CFG")          # "cfg,splits" override for tuning sweeps
_FORCE_CFG = tuple(int(v) for v in _env.split(",")) if _env else None


def _lib():
    from . import native
    lib = native.load()
    if not _sig_done[0]:
        V, I, LL, F = _c.c_void_p, _c.c_int, _c.c_longlong, _c.c_float
        lib.dl4j_gemm_plan.argtypes = [I, I, I, I, _c.POINTER(I), _c.POINTER(I)]
        lib.dl4j_gemm_plan.restype = LL
        lib.dl4j_gemm.argtypes = [I, I, I, I, I, I, V, LL, I, LL, V, LL, I, LL, V, LL, LL, F, F, V, I, I, V, I, I, V, V, I,
                                  V]
        lib.dl4j_gemm.restype = I
        lib.dl4j_gemm_simple.argtypes = [I, I, I, I, I, I, V, LL, LL, LL, V, LL, LL, LL, V, LL, LL, F, F, V, I, I, V, V]
        lib.dl4j_gemm_simple.restype = I
        lib.dl4j_gemm_f32_plan.argtypes = [I, I, I, I, _c.POINTER(I), _c.POINTER(I)]
        lib.dl4j_gemm_f32_plan.restype = LL
        lib.dl4j_gemm_f32.argtypes = [I, I, I, I, I, I, V, LL, LL, LL, V, LL, LL, LL, V, LL, LL, F, F, V, I, I, V, I, I,
                                      V, V]
        lib.dl4j_gemm_f32.restype = I
        _sig_done[0] = True
    return lib


_TUNED = {}                                            # problem key -> (cfg, splits), filled by _autotune
_TUNE = os.environ.get("DL4J_AMD_GEMM_TUNE", "1") == "1"
_TUNE_LOG = os.environ.get("DL4J_AMD_GEMM_TUNE_LOG", "0") == "1"   # print every autotuned shape's candidate times
# Opt-in (DL4J_AMD_GEMM_LIB=1): hipBLASLt (torch.mm / addmm / bmm on the same stream, plus an in-tree elementwise
# kernel for an activation epilogue) as one more autotuner candidate, used where it measured faster. Off by default:
# every product runs on the in-tree MFMA kernels, and a library pick is counted as a helper fallback
# (ops/fallback.py, helperCountFail()).
_LIB = os.environ.get("DL4J_AMD_GEMM_LIB", "0") == "1"
LIB_CFG = (-2, 1)
STREAM_CFG = (10, 1)     # csrc/gemm_stream.hip: persistent loader-wave kernel for tall short-K (1x1-conv) products
_F32_FORCE = None        # tests: True / False pins fp32 products to the library / the exact-fp32 kernel


def _plan(lib, M, N, K, batch):
    cfg, sp = _c.c_int(-1), _c.c_int(0)
    lib.dl4j_gemm_plan(M, N, K, batch, _c.byref(cfg), _c.byref(sp))
    return cfg.value, sp.value


def _candidates(M, N, K, batch, default):
    c = [default]
    t256 = ((M + 255) // 256) * ((N + 255) // 256) * batch
    t128 = ((M + 127) // 128) * ((N + 127) // 128) * batch
    splits = (1, 2, 3, 4, 6, 8, 12, 16, 24, 32, 48, 64, 96, 128, 192, 256)
    if K % 64 == 0:
        c += [(4, s) for s in splits if s == 1 or (batch == 1 and K // s >= 512 and t256 * s <= 1024)]
    c += [(x, 1) for x in (0, 1, 2, 3, 5, 6, 7, 8, 9)]
    if batch == 1 and M % 128 == 0 and N % 64 == 0 and K % 64 == 0 and K // 64 in (1, 2, 4, 8):
        c.append(STREAM_CFG)      # persistent streaming kernel (refuses, -4, layouts / epilogues it lacks)
    if batch == 1:
        # small output grids (e.g. the LSTM's [256 x 1024] weight gradients over K = T*mb = 1600) need deep split-K
        # to fill the CUs: down to 128-deep K slices when the tile grid is under a quarter of the chip
        kmin = 128 if t128 * 4 <= 256 else 512
        c += [(x, s) for x in (1, 2, 3, 5) for s in splits[1:] if K // s >= kmin and t128 * s <= 2048]
        # deep-ring 128x128 tiles (cfg 6 / 7): one block per CU, so splits that keep the grid near 1-2 waves of CUs
        c += [(x, s) for x in (6, 7) for s in splits[1:] if K // s >= 256 and 128 <= t128 * s <= 768]
    seen, out = set(), []
    for x in c:
        if x not in seen:
            seen.add(x)
            out.append(x)
    return out


def _autotune(launch, c_t, M, N, K, batch, default, splits_ok=True, lib=False, zz=None):
    """First eager call of a problem shape: time every kernel configuration (tile shape x split-K; plus the library
    GEMM when ``lib``) on a scratch destination and keep the fastest. ``zz``: the call's pre-activation buffer, so
    every candidate is timed with its epilogue (a forward activation rewrites it, dgelu reads it). Never runs while a
    HIP graph is being captured; the cost-model plan is used there."""
    from .timing import gpu_time
    tmp = torch.empty_strided(c_t.size(), c_t.stride(), dtype=c_t.dtype, device=c_t.device)
    best, best_t = default, None
    log = [] if _TUNE_LOG else None
    for cand in _candidates(M, N, K, batch, default) + ([LIB_CFG] if lib else []):
        if cand[1] > 1 and not splits_ok:
            continue
        if launch(cand[0], cand[1], tmp, 0.0, zz) != 0:
            continue
        # GPU-side time (stream parked during the enqueue): small GEMMs are shorter than the host launch path
        t = gpu_time(lambda: launch(cand[0], cand[1], tmp, 0.0, zz), reps=tunedb.reps(3), warmup=0)
        if log is not None:
            log.append((t, cand))
        if best_t is None or t < best_t:
            best, best_t = cand, t
    if log:
        log.sort()
        print(f"[gemm-tune] M={M} N={N} K={K} batch={batch} out={c_t.dtype} zz={zz is not None} best={best} " +
              " ".join(f"{c[0]}/{c[1]}:{t * 1e3:.1f}" for t, c in log[:8]), flush=True)
    return best


def _p(t):
    return None if t is None else _c.c_void_p(t.data_ptr())


def _a_layout(t):
    """(kc, ld) for an [M, K] operand view, or None when neither dimension is unit-stride."""
    M, K = t.shape[-2], t.shape[-1]
    s0, s1 = t.stride(-2), t.stride(-1)
    if s1 == 1 or K == 1:
        return True, (s0 if M > 1 else (K + 7) // 8 * 8)
    if s0 == 1 or M == 1:
        return False, (s1 if K > 1 else (M + 7) // 8 * 8)
    return None


def _b_layout(t):
    """(kc, ld) for a [K, N] operand view: kc=True when K is the unit-stride dimension."""
    K, N = t.shape[-2], t.shape[-1]
    s0, s1 = t.stride(-2), t.stride(-1)
    if s0 == 1 or K == 1:
        return True, (s1 if N > 1 else (K + 7) // 8 * 8)
    if s1 == 1 or N == 1:
        return False, (s0 if K > 1 else (N + 7) // 8 * 8)
    return None


def _fast_ok(t, lay, K, is_a):
    """Mirror of dl4j_gemm's addressing requirements for one operand (16-byte DMA chunks). A K-contiguous operand
    with K % 8 != 0 qualifies when it is a view of a buffer whose columns K..K8-1 are zeros (``kz_view``)."""
    if lay is None or t.data_ptr() % 16 or lay[1] % 8:
        return False
    if t.dim() == 3 and t.stride(0) % 8:
        return False
    if lay[0] and K % 8:
        K8 = (K + 7) // 8 * 8
        return getattr(t, "_dl4j_kz", 0) >= K8 and lay[1] >= K8
    return True


def kz_view(buf, K):
    """[.., K] view of the [.., K8] buffer ``buf`` whose columns K..K8-1 are zero: the GEMM then reads the operand in
    place (its 16-byte chunk past K only meets zeros) instead of making a padded copy."""
    v = buf[..., :K]
    v._dl4j_kz = buf.shape[-1]
    return v


def _pad_kc(t, K, K8):
    """[.., R, K] operand -> contiguous [.., R, K8] copy with zeros in columns K..K8-1 (one strided-copy launch on the
    GPU)."""
    if t.is_cuda:
        from . import nd4j_kernels as NK
        r = NK.cast_pad_last(t, t.dtype, K8)
        if r is not None:
            return r
    p = torch.zeros(t.shape[:-1] + (K8,), dtype=t.dtype, device=t.device)
    p[..., :K].copy_(t)
    return p


def _torch_mmul(a, b, out, bias, bias_dim, act, alpha, beta, out_dtype, z):
    cd = a.dtype if a.dtype in (torch.float64, torch.float32) else torch.float32
    r = torch.matmul(a.to(cd), b.to(cd))
    if alpha != 1.0:
        r = r * alpha
    if bias is not None:
        r = r + (bias.to(cd).reshape(1, -1) if bias_dim == 1 else bias.to(cd).reshape(-1, 1))
    if beta != 0.0 and out is not None:
        r = r + beta * out.to(cd)
    if act == "dgelu":
        r = r * _dgelu_ref(z.to(cd)) if z is not None else r
    else:
        if z is not None:
            z.copy_(r)
        r = _torch_act(r, act)
    if out is not None:
        out.copy_(r)
        return out
    from ..memory import arena
    if arena.current() is not None:
        return arena.empty(r.shape, out_dtype, r.device).copy_(r)
    return r.to(out_dtype)


def _dgelu_ref(z):
    cdf = 0.5 * (1.0 + torch.erf(z * 0.7071067811865476))
    pdf = torch.exp(-0.5 * z * z) * 0.3989422804014327
    return cdf + z * pdf


def _torch_act(r, act):
    if act in (None, "identity"):
        return r
    if act == "relu":
        return torch.relu(r)
    if act == "tanh":
        return torch.tanh(r)
    if act == "sigmoid":
        return torch.sigmoid(r)
    if act == "gelu":
        return torch.nn.functional.gelu(r)
    raise ValueError(act)


def mmul(a, b, out=None, bias=None, bias_dim=1, act=None, alpha=1.0, beta=0.0, out_dtype=None, z=None, stats=None,
         stats_tag=None):
    """``out = act(alpha * a @ b + bias + beta * out)``; returns ``out`` (allocated row-major when None).

    a: [M, K] or [B, M, K]; b: [K, N] or [B, K, N]; bias: [N] (bias_dim=1) or [M] (bias_dim=0);
    z: optional tensor like ``out`` receiving the pre-activation (act="dgelu": the pre-activation that is READ, out =
    (a @ b) * gelu'(z)); out_dtype defaults to a.dtype.
    stats: optional fp32 [3, P, N] tensor (P = ceil(M/64)) receiving per-64-row BatchNorm partial statistics of the
    bf16 output (conv -> BN fusion; 8-phase kernel). With the BN-backward epilogue armed (ops/native.py bnb_armed)
    the buffer is [2, P, N] and receives the BN backward sums instead; stats_tag keeps its tuned tile separate.
    """
    if b.dtype != a.dtype:
        # mixed operands: compute in the 16-bit type (fp32 accumulation) rather than promoting to the exact-fp32 path
        lo = [t for t in (a.dtype, b.dtype) if t in (torch.bfloat16, torch.float16)]
        ct = lo[0] if lo and a.is_cuda else a.dtype
        a, b = a.to(ct), b.to(ct)
    out_dtype = out.dtype if out is not None else (out_dtype or a.dtype)
    if not use_native(a, "gemm"):
        return _torch_mmul(a, b, out, bias, bias_dim, act, alpha, beta, out_dtype, z)
    if a.dtype not in _DT or out_dtype not in _DT or (z is not None and z.dtype != out_dtype):
        fallback.record("gemm", f"dtype {a.dtype}->{out_dtype}")
        return _torch_mmul(a, b, out, bias, bias_dim, act, alpha, beta, out_dtype, z)
    batched = a.dim() == 3 or b.dim() == 3
    if batched:
        if a.dim() == 2:
            a = a.unsqueeze(0).expand(b.shape[0], -1, -1)
        if b.dim() == 2:
            b = b.unsqueeze(0).expand(a.shape[0], -1, -1)
        batch = a.shape[0]
    else:
        batch = 1
    M, K = a.shape[-2], a.shape[-1]
    N = b.shape[-1]
    if b.shape[-2] != K:
        raise ValueError(f"mmul shape mismatch {tuple(a.shape)} x {tuple(b.shape)}")
    if out is None:
        from ..memory import arena
        out = arena.empty(((batch,) if batched else ()) + (M, N), out_dtype, a.device)
        if beta != 0.0:
            raise ValueError("beta != 0 needs an existing out")
    if M == 0 or N == 0:
        return out
    if K == 0:
        out.zero_() if beta == 0.0 else out.mul_(beta)
        return out
    bias_in = None
    if bias is not None:
        # the operand-dtype copy of the bias (a library GEMM's epilogue needs it): the bias itself, or the 16-bit
        # shadow the network / SameDiff attached to an fp32 master parameter
        bias_in = bias if bias.dtype == a.dtype else getattr(bias, "_dl4j_shadow", None)
        bias_in = None if bias_in is None else bias_in.reshape(-1)
        bias = bias.reshape(-1)
        if bias.dtype != torch.float32 or not bias.is_contiguous():
            bias = bias.to(torch.float32).contiguous()
    bmode = 0 if bias is None else (1 if bias_dim == 1 else 2)
    c_t = out
    swap = False
    if out.stride(-1) == 1 or N == 1:
        ldc = out.stride(-2) if M > 1 else N
    elif out.stride(-2) == 1 or M == 1:
        swap = True
        ldc = out.stride(-1) if N > 1 else M
    else:
        c_t = torch.empty(out.shape, dtype=out_dtype, device=a.device)
        ldc = N
        if beta != 0.0:
            c_t.copy_(out)
    if z is not None and (z.shape != out.shape or z.stride() != c_t.stride()):
        fallback.record("gemm", "pre-activation layout differs from output")
        return _torch_mmul(a, b, out, bias, bias_dim, act, alpha, beta, out_dtype, z)
    la, lb = _a_layout(a), _b_layout(b)
    if a.dtype != torch.float32 and not (_fast_ok(a, la, K, True) and _fast_ok(b, lb, K, False)):
        # odd K / leading dimensions: zero-padded K-contiguous copies (usually a small operand such as a one-hot
        # input) keep the product on the MFMA LDS-DMA kernel instead of the scalar-load generic one
        K8 = (K + 7) // 8 * 8
        if not _fast_ok(a, la, K, True):
            a = _pad_kc(a, K, K8)[..., :K]
            la = (True, K8)
        if not _fast_ok(b, lb, K, False):
            b = _pad_kc(b.transpose(-1, -2), K, K8)[..., :K].transpose(-1, -2)
            lb = (True, K8)
    # K-contiguous operands with K % 8 != 0 are zero-padded to K8 here (flag 2 for dl4j_gemm); M/N-contiguous ones
    # read rows >= K from the kernel's zero page
    kzf = lambda lay: (2 if lay is not None and lay[0] and K % 8 else 0)  # noqa: E731
    sA = a.stride(0) if batched else 0
    sB = b.stride(0) if batched else 0
    sC = c_t.stride(0) if batched else 0
    lib = _lib()
    from .native import _stream
    actc = ACT[act]
    if swap:
        # C^T [N, M] = B^T A^T
        Mx, Nx = N, M
        A_, B_ = b, a
        la_, lb_ = lb, la
        sA_, sB_ = sB, sA
        bmode = {0: 0, 1: 2, 2: 1}[bmode]
    else:
        Mx, Nx = M, N
        A_, B_ = a, b
        la_, lb_ = la, lb
        sA_, sB_ = sA, sB
    in_dt = _DT[a.dtype]
    rc = -1
    if in_dt != 0 and la_ is not None and lb_ is not None:
        def launch(cfg, sp, dst, bt, zz, ts=None):
            ws = torch.empty(Mx * Nx * sp, dtype=torch.float32, device=a.device) if sp > 1 else None
            return lib.dl4j_gemm(in_dt, _DT[out_dtype], Mx, Nx, K, batch, _p(A_), la_[1], int(la_[0]) | kzf(la_),
                                 sA_, _p(B_), lb_[1], int(lb_[0]) | kzf(lb_), sB_, _p(dst), ldc, sC, float(alpha), bt, _p(bias), bmode, actc,
                                 _p(zz), cfg, sp, _p(ws), _p(ts), 0 if ts is None else ts.shape[1], _stream())

        key = (Mx, Nx, K, batch, in_dt, _DT[out_dtype], la_[0], lb_[0], la_[1] % 64 == 0, lb_[1] % 64 == 0)
        if stats is not None:
            if swap or batch != 1:
                raise ValueError("GEMM BatchNorm statistics need a row-major, unbatched destination")
            kst = key + ("stats", stats_tag)
            cfg = (_FORCE_CFG[0], 1) if _FORCE_CFG is not None else _TUNED.get(kst)
            from_db = False
            if cfg is None:
                cfg = tunedb.lookup("gemm", kst)
                if cfg is not None:
                    _TUNED[kst] = cfg
                    from_db = True
                else:
                    cfg = (4, 1) if K % 64 == 0 else (2, 1)
                    if _TUNE and not torch.cuda.is_current_stream_capturing():
                        cfg = _autotune(lambda c_, s_, d_, bt_, zz_: launch(c_, s_, d_, bt_, zz_, stats), c_t, Mx, Nx,
                                        K, batch, cfg, splits_ok=False)
                        _TUNED[kst] = cfg
                        tunedb.record("gemm", kst, cfg)
            rc = launch(cfg[0], 1, c_t, float(beta), z, stats)
            if rc != 0 and from_db:
                # a recorded choice this build refuses: drop it and take the planner's default configuration
                tunedb.forget("gemm", kst)
                cfg = (4, 1) if K % 64 == 0 else (2, 1)
                _TUNED[kst] = cfg
                rc = launch(cfg[0], 1, c_t, float(beta), z, stats)
            if rc != 0:
                raise RuntimeError(f"HIP gemm (stats) failed with code {rc}")
            if c_t is not out:
                out.copy_(c_t)
            return out
        libmm = None if (bias is not None and bias_in is None) else \
            _lib_gemm(a, b, c_t, swap, batched, bias_in, bias_dim, act, alpha, beta, z, out_dtype)
        if libmm is not None:
            key = key + ("lib", bias_in is not None, beta != 0.0, act, z is not None)
            kern = launch

            def launch(cfg, sp, dst, bt, zz, ts=None):
                return libmm(dst, bt) if cfg == LIB_CFG[0] else kern(cfg, sp, dst, bt, zz, ts)
        from_db = False
        if _FORCE_CFG is not None:
            cfg = _FORCE_CFG
        else:
            cfg = _TUNED.get(key)
            if cfg is None:
                cfg = tunedb.lookup("gemm", key)
                if cfg is not None:
                    _TUNED[key] = cfg
                    from_db = True
                else:
                    cfg = _plan(lib, Mx, Nx, K, batch)
                    if _TUNE and not torch.cuda.is_current_stream_capturing():
                        cfg = _autotune(launch, c_t, Mx, Nx, K, batch, cfg, lib=libmm is not None, zz=z)
                        _TUNED[key] = cfg
                        tunedb.record("gemm", key, cfg)
        if cfg == LIB_CFG:
            fallback.record("gemm", "library GEMM (hipBLASLt) picked by the autotuner (DL4J_AMD_GEMM_LIB=1)")
        rc = launch(cfg[0], cfg[1], c_t, float(beta), z)
        if rc != 0 and from_db:
            # a recorded choice this build / device refuses: drop it, re-plan (the autotuner re-times next call)
            tunedb.forget("gemm", key)
            _TUNED.pop(key, None)
            cfg = _plan(lib, Mx, Nx, K, batch)
            rc = launch(cfg[0], cfg[1], c_t, float(beta), z)
    if rc == -1:
        # exact-fp32 MFMA kernel: any dtype / strides
        if swap:
            sam, sak = A_.stride(-1), A_.stride(-2)
            sbk, sbn = B_.stride(-1), B_.stride(-2)
        else:
            sam, sak = A_.stride(-2), A_.stride(-1)
            sbk, sbn = B_.stride(-2), B_.stride(-1)

        # tiled split-K exact-fp32 kernel (64/128 tiles, slabs from torch's allocator; reduce applies the epilogue)
        tile, nsp = _c.c_int(0), _c.c_int(1)
        wsb = lib.dl4j_gemm_f32_plan(Mx, Nx, K, batch, _c.byref(tile), _c.byref(nsp))
        ws32 = torch.empty(wsb // 4, dtype=torch.float32, device=c_t.device) if wsb > 0 else None

        def simple(dst, bt):
            return lib.dl4j_gemm_f32(in_dt, _DT[out_dtype], Mx, Nx, K, batch, _p(A_), sam, sak, sA_, _p(B_), sbk,
                                     sbn, sB_, _p(dst), ldc, sC, float(alpha), bt, _p(bias), bmode, actc, _p(z),
                                     tile.value, nsp.value, _p(ws32), _stream())
        run = simple
        if in_dt == 0 and not (bias is not None and bias_in is None):
            # fp32 operands with DL4J_AMD_GEMM_LIB=1: the fp32 library GEMM (exact fp32, no TF32) is a second
            # candidate, timed per shape like the 16-bit configurations (counted as a fallback when picked)
            libmm = _lib_gemm(a, b, c_t, swap, batched, bias_in, bias_dim, act, alpha, beta, z, out_dtype)
            if libmm is not None:
                k32 = ("f32", Mx, Nx, K, batch, swap, sam, sak, sbk, sbn, ldc, bias_in is not None, beta != 0.0, act,
                       z is not None)
                use_lib = _TUNED.get(k32) if _F32_FORCE is None else _F32_FORCE
                if use_lib is None:
                    use_lib = False
                    if _TUNE and not torch.cuda.is_current_stream_capturing():
                        from .timing import gpu_time
                        tmp = torch.empty_strided(c_t.size(), c_t.stride(), dtype=c_t.dtype, device=c_t.device)
                        if simple(tmp, 0.0) == 0 and libmm(tmp, 0.0) == 0:
                            use_lib = gpu_time(lambda: libmm(tmp, 0.0), reps=3, warmup=0) < \
                                gpu_time(lambda: simple(tmp, 0.0), reps=3, warmup=0)
                        _TUNED[k32] = use_lib
                if use_lib:
                    run = libmm
                    fallback.record("gemm", "fp32 library GEMM (hipBLASLt) picked by the autotuner")
        rc = run(c_t, float(beta))
    if rc != 0:
        raise RuntimeError(f"HIP gemm failed with code {rc} (M={M} N={N} K={K} batch={batch})")
    if c_t is not out:
        out.copy_(c_t)
    return out


def _lib_gemm(a, b, c_t, swap, batched, bias, bias_dim, act, alpha, beta, z, out_dtype):
    """A launcher ``(dst, beta) -> 0`` running the product as one hipBLASLt call through torch on the current stream
    (plus, for an activation epilogue, one in-tree elementwise kernel over the result), or None when the problem needs
    an epilogue only the in-tree GEMM has (a row bias, alpha != 1, beta with an activation, fp32 output combined with
    a bias / beta / batch) or its destination is not a dense matrix.
    Activations: ``act(z)`` with the pre-activation kept in ``z`` when given (the library writes z, the elementwise
    kernel reads it); ``dgelu``: out = (a @ b) * gelu'(z), applied in place on the library result."""
    if not _LIB or alpha != 1.0 or a.dtype not in (torch.bfloat16, torch.float16, torch.float32) or b.dtype != a.dtype:
        return None
    act = None if act == "identity" else act
    if act not in (None, "relu", "tanh", "sigmoid", "gelu", "dgelu") or (act is not None and (beta != 0.0 or batched)):
        return None
    if (act == "dgelu" and z is None) or (z is not None and act is None):
        return None
    wide = out_dtype == torch.float32 and a.dtype != torch.float32     # 16-bit operands, fp32 result (weight grads)
    if out_dtype != a.dtype and not (wide and bias is None and beta == 0.0 and not batched and act is None):
        return None
    if bias is not None and (bias.dtype != a.dtype or bias_dim != 1 or swap or batched or beta != 0.0):
        return None
    dstv = (lambda d: d.mT) if swap else (lambda d: d)                 # noqa: E731
    if not dstv(c_t).is_contiguous() or (z is not None and not dstv(z).is_contiguous()):
        return None
    A_, B_ = (b.mT, a.mT) if swap else (a, b)
    if act is not None:
        from . import nd4j_kernels as NK
        if not NK.ok(c_t):
            return None

    def run(dst, bt):
        d = dstv(dst)
        pre = dstv(z) if (z is not None and act != "dgelu") else d
        if wide:
            torch.mm(A_, B_, out_dtype=torch.float32, out=d)
        elif bias is not None:
            torch.addmm(bias, A_, B_, out=pre)
        elif bt == 0.0:
            (torch.bmm if batched else torch.mm)(A_, B_, out=pre)
        else:
            (d.baddbmm_ if batched else d.addmm_)(A_, B_, beta=bt)
        if act == "dgelu":
            r = native_gelu_(dstv(z), d)
            if r != 0:
                return r
        elif act == "gelu":                     # the vectorized GELU kernel (the generic transform is ~3x slower)
            r = native_gelu_(pre, None, out=d)
            if r != 0:
                return r
        elif act is not None:
            if NK.transform(pre, act, out=d) is None:
                return -1
        return 0
    return run


def native_gelu_(z, dy, out=None):
    """On the in-tree GELU kernel (csrc/activations.hip): dy *= gelu'(z) in place, or with dy None out = gelu(z);
    0 or an error code."""
    from .native import _stream
    from . import transformer_native as TN
    d = _DT.get(z.dtype)
    dst = dy if dy is not None else out
    if d is None or not (z.is_contiguous() and dst.is_contiguous()) or dst.dtype != z.dtype:
        return -1
    TN.native.register_sig("dl4j_gelu", [_c.c_int, _c.c_void_p, _c.c_void_p, _c.c_void_p, _c.c_longlong,
                                         _c.c_void_p])
    return _lib().dl4j_gelu(d, _p(z), _p(dy), _p(dst), z.numel(), _c.c_void_p(_stream()))


def bias_vec(b):
    """``b`` as a 1-D bias that keeps its 16-bit shadow (``_dl4j_shadow``, the library GEMM's bias operand) — a plain
    ``reshape(-1)`` returns a new tensor object without the attribute."""
    if b is None:
        return None
    sh = getattr(b, "_dl4j_shadow", None)
    v = b.reshape(-1)
    if sh is not None and v is not b:
        v._dl4j_shadow = sh.reshape(-1)
    return v


def linear(x, W, b=None, act=None, z=None, out_dtype=None):
    """x [M, K] @ W [K, N] + b — DL4J preOutput (BaseLayer.java:334-336) with a fused bias / activation epilogue."""
    return mmul(x, W, bias=b, act=act, z=z, out_dtype=out_dtype)

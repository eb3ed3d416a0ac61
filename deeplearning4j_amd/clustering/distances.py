"""Distance functions and GEMM-based brute-force k-NN.

Names follow the reference (VPTree.distance: euclidean, manhattan, cosinesimilarity, cosinedistance, dot, hamming,
jaccard). Euclidean/cosine/dot pairwise matrices are one GEMM (|x|^2 + |y|^2 - 2 x.y), chunked over queries so a
[chunk, N] tile stays in HBM; manhattan/hamming/jaccard use broadcast reductions.
"""
import torch

DISTANCES = {"euclidean": 0, "manhattan": 1, "cosinedistance": 2, "cosinesimilarity": 3, "dot": 4, "hamming": 5,
             "jaccard": 6}

# similarity functions: larger is closer (the reference inverts them with ``invert``)
SIMILARITIES = {"cosinesimilarity", "dot"}


def pairwise(q, x, fn="euclidean"):
    """[nq, N] distance matrix between rows of q and rows of x."""
    q = q.float()
    x = x.float()
    if fn == "euclidean":
        d2 = (q * q).sum(1, keepdim=True) + (x * x).sum(1).unsqueeze(0) - 2.0 * (q @ x.t())
        return d2.clamp_min(0).sqrt()
    if fn in ("cosinesimilarity", "cosinedistance"):
        qn = q / q.norm(dim=1, keepdim=True).clamp_min(1e-30)
        xn = x / x.norm(dim=1, keepdim=True).clamp_min(1e-30)
        s = qn @ xn.t()
        return s if fn == "cosinesimilarity" else 1.0 - s
    if fn == "dot":
        return q @ x.t()
    if fn == "manhattan":
        return torch.cdist(q, x, p=1)
    if fn == "hamming":
        return (q.unsqueeze(1) != x.unsqueeze(0)).float().mean(-1)
    if fn == "jaccard":
        mn = torch.minimum(q.unsqueeze(1), x.unsqueeze(0)).sum(-1)
        mx = torch.maximum(q.unsqueeze(1), x.unsqueeze(0)).sum(-1)
        return torch.where(mx > 0, 1.0 - mn / mx.clamp_min(1e-30), torch.zeros_like(mx))
    raise ValueError(f"unknown distance function {fn!r}")


def knn_bruteforce(x, queries, k, fn="euclidean", invert=False, chunk=4096):
    """Exact k-NN by blocked distance GEMM + top-k. Returns (indices [nq,k] int64, distances [nq,k]),
    ascending by (inverted) distance."""
    k = min(k, x.shape[0])
    outs_i, outs_d = [], []
    sign = -1.0 if (invert or fn in SIMILARITIES) else 1.0
    for s in range(0, queries.shape[0], chunk):
        d = pairwise(queries[s:s + chunk], x, fn) * sign
        v, i = torch.topk(d, k, dim=1, largest=False)
        outs_i.append(i)
        outs_d.append(v * sign if not invert else v)
    return torch.cat(outs_i), torch.cat(outs_d)

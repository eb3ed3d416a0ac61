"""BERT input-embedding kernels (csrc/nn_misc.hip bert_embed_*) against a plain fp32 torch reference: the forward sum
of word / position / type rows, and the position / type gradients (deterministic column sums) with the word rows'
scatter-add, including 'f'-ordered gradient views and position tables longer than the sequence."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16, torch.float32])
@pytest.mark.parametrize("B,T,E,Tmax", [(8, 128, 768, 512), (3, 7, 64, 7), (2, 33, 136, 40)])
def test_bert_embed_forward(dtype, B, T, E, Tmax):
    from deeplearning4j_amd.ops import nn_misc
    g = torch.Generator().manual_seed(B * T + E)
    V = 1000
    Ww = torch.randn(V, E, generator=g).cuda().to(dtype)
    Wp = torch.randn(Tmax, E, generator=g).cuda().to(dtype)
    Wt = torch.randn(2, E, generator=g).cuda().to(dtype)
    idx = torch.randint(0, V, (B, T), generator=g).cuda()
    out = nn_misc.bert_embed_forward(Ww, Wp, Wt, idx)
    assert out is not None
    ref = Ww.float()[idx.reshape(-1)] + Wp.float()[:T].repeat(B, 1) + Wt.float()[0]
    tol = 1e-6 if dtype == torch.float32 else (1e-2 if dtype == torch.bfloat16 else 2e-3)
    torch.testing.assert_close(out.float(), ref, rtol=tol, atol=tol * 4)


@pytest.mark.parametrize("f_order", [False, True])
@pytest.mark.parametrize("B,T,E,Tmax", [(8, 128, 768, 512), (2, 33, 136, 33)])
def test_bert_embed_backward(f_order, B, T, E, Tmax):
    from deeplearning4j_amd.ops import nn_misc
    g = torch.Generator().manual_seed(T + E)
    de = torch.randn(B * T, E, generator=g).cuda().to(torch.bfloat16)
    ntype = 2

    def view(r, c):
        if f_order:
            return torch.full((c, r), 7.0, device="cuda").t()     # column-major view, stale contents
        return torch.full((r, c), 7.0, device="cuda")
    gpos, gtype = view(Tmax, E), view(ntype, E)
    assert nn_misc.bert_embed_backward_pt(de, gpos, gtype, B, T)
    d = de.float().reshape(B, T, E)
    ref_pos = torch.zeros(Tmax, E, device="cuda")
    ref_pos[:T] = d.sum(0)
    ref_type = torch.zeros(ntype, E, device="cuda")
    ref_type[0] = d.sum((0, 1))
    torch.testing.assert_close(gpos, ref_pos, rtol=1e-5, atol=1e-4)
    torch.testing.assert_close(gtype, ref_type, rtol=1e-5, atol=1e-3)
    # deterministic: a second call writes the same bits
    gpos2, gtype2 = view(Tmax, E), view(ntype, E)
    assert nn_misc.bert_embed_backward_pt(de, gpos2, gtype2, B, T)
    assert torch.equal(gpos, gpos2) and torch.equal(gtype, gtype2)


def test_bert_embedding_layer_gradients_match_fp32():
    """The BertBase embedding layer's word / position / type gradients from the in-tree path vs an fp32 autograd
    reference of the same sum + LayerNorm."""
    from deeplearning4j_amd.models import BertBase
    from deeplearning4j_amd.nn.conf import DataType
    torch.manual_seed(0)
    net = BertBase(numLabels=2, inputShape=[16], layers=1, dataType=DataType.BFLOAT16).init(device=torch.device("cuda", 0))
    impls = [impl for _, _, impl, _ in net._layer_offsets]
    emb = next(i for i in impls if type(i).__name__ == "BertEmbeddingLayerImpl")
    B, T = 4, 16
    idx = torch.randint(0, 30522, (B, T)).cuda()
    idx[0, :4] = idx[1, :4]                                      # repeated tokens: scatter-add must sum them
    y = emb.activate(idx, training=True)
    eps = torch.randn_like(y.float()).to(y.dtype)
    for k in ("Wword", "Wpos", "Wtype"):
        emb.grads[k].fill_(0.0)
    emb.backpropGradient(eps)
    Ww = emb.params["Wword"].detach().float().clone().requires_grad_(True)
    Wp = emb.params["Wpos"].detach().float().clone().requires_grad_(True)
    Wt = emb.params["Wtype"].detach().float().clone().requires_grad_(True)
    e = Ww[idx.reshape(-1)] + Wp[:T].repeat(B, 1) + Wt[0]
    ln = torch.nn.functional.layer_norm(e, (e.shape[1],), emb.params["lng"].float().reshape(-1),
                                        emb.params["lnb"].float().reshape(-1),
                                        eps=emb.conf.layerNormEps)
    ln.backward(eps.permute(0, 2, 1).reshape(B * T, -1).float())
    for k, ref in (("Wword", Ww.grad), ("Wpos", Wp.grad), ("Wtype", Wt.grad)):
        got = emb.grads[k].float()
        cos = torch.nn.functional.cosine_similarity(got.reshape(-1), ref.reshape(-1), dim=0).item()
        assert cos > 0.999, (k, cos)
        assert abs(got.norm().item() / ref.norm().item() - 1) < 0.02, k

"""North-star model zoo on CPU (tiny configs): BERT MLM under SSP(1), Llama with 1-bit push
(gloo world 2), DLRM with sharded sparse tables + row-wise Adagrad (gloo world 2), ResNet
bottleneck path.  Full-size parameter counts are checked on the meta device."""
import torch
import torch.nn.functional as F

from tests import dist_util


def test_param_counts_match_published():
    from ps_amd.models.resnet import resnet50
    from ps_amd.models.transformer import BertForMLM, LlamaConfig, LlamaForCausalLM, param_count

    with torch.device("meta"):
        assert abs(param_count(BertForMLM()) / 1e6 - 109.5) < 0.5  # BERT-base (tied decoder)
        assert abs(param_count(LlamaForCausalLM(LlamaConfig.llama3_8b())) / 1e9 - 8.03) < 0.01
    assert param_count(resnet50()) == 25557032


def test_bert_tiny_ssp_learns():
    from ps_amd.models.transformer import BertConfig, BertForMLM, mlm_batch
    from ps_amd.parallel.colocated import ColocatedPS
    from ps_amd.parallel.updaters import AdamUpdater

    torch.manual_seed(0)
    m = BertForMLM(BertConfig(vocab=300, hidden=32, layers=2, heads=4, ffn=64, max_pos=32, dropout=0.0))
    ps = ColocatedPS(m, AdamUpdater(3e-3, bias_correction="step"), staleness=1, bucket_mb=0.05)
    ids, labels = mlm_batch(16, 16, vocab=300, seed=0)
    losses = []
    for _ in range(30):
        loss = m(ids, labels)
        loss.backward()
        ps.finish_step()
        losses.append(loss.item())
    assert losses[-1] < losses[0] - 1.0


def test_bert_masked_positions_head_matches_dense_head():
    """The sparse-prediction head (masked_lm_positions) computes the same loss and gradients
    as the dense head with ignore_index -- it only skips the unmasked rows."""
    from ps_amd.models.transformer import BertConfig, BertForMLM, mlm_batch

    torch.manual_seed(0)
    m = BertForMLM(BertConfig(vocab=300, hidden=32, layers=2, heads=4, ffn=64, max_pos=32, dropout=0.0))
    ids, labels, pos = mlm_batch(8, 20, vocab=300, seed=1, with_positions=True)
    assert pos.shape == (8, 3) and bool((labels != -100).sum(1).eq(3).all())
    l_dense = m(ids, labels)
    g_dense = torch.autograd.grad(l_dense, list(m.parameters()))
    l_sparse = m(ids, labels, pos)
    g_sparse = torch.autograd.grad(l_sparse, list(m.parameters()))
    torch.testing.assert_close(l_sparse, l_dense)
    for a, b in zip(g_sparse, g_dense):
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-6)


def _llama_body(tp):
    from ps_amd.models.transformer import LlamaConfig, LlamaForCausalLM
    from ps_amd.parallel.colocated import ColocatedPS
    from ps_amd.parallel.updaters import AdamUpdater

    torch.manual_seed(0)
    m = LlamaForCausalLM(LlamaConfig.tiny(), checkpointing=True)
    ps = ColocatedPS(m, AdamUpdater(3e-3, bias_correction="step"), tp, compress="onebit", bucket_mb=0.1)
    g = torch.Generator().manual_seed(tp.rank)
    ids = torch.randint(0, 512, (4, 32), generator=g)
    losses = []
    for _ in range(15):
        loss = m(ids, ids)
        loss.backward()
        ps.finish_step()
        losses.append(loss.item())
    return losses, m.lm_head.weight.detach().clone()


def test_llama_tiny_onebit_world2():
    res = dist_util.run(_llama_body, 2)
    assert res[0][0][-1] < res[0][0][0]
    torch.testing.assert_close(res[0][1], res[1][1])  # replicas identical after compressed rounds


def _dlrm_body(tp):
    from ps_amd.models.dlrm import DLRM, dlrm_batch
    from ps_amd.parallel.colocated import ColocatedPS
    from ps_amd.parallel.updaters import AdagradUpdater

    torch.manual_seed(0)
    rows = [500] * 4
    m = DLRM(dense_in=13, table_rows=rows, dim=16, bottom=(32,), top=(32, 16), transport=tp)
    ps = ColocatedPS(m, AdagradUpdater(0.05, 1e-8), tp, bucket_mb=0.05)
    dense, sparse, y = dlrm_batch(256, rows, seed=tp.rank)
    losses = []
    for _ in range(20):
        loss = F.binary_cross_entropy_with_logits(m(dense, sparse), y)
        loss.backward()
        m.push_sparse()
        ps.finish_step()
        losses.append(loss.item())
    probe = m.emb.table.pull_keys(torch.tensor([0, 1, 2, 600, 1999]))
    return losses, probe


def test_dlrm_sharded_world2():
    res = dist_util.run(_dlrm_body, 2)
    assert res[0][0][-1] < res[0][0][0]
    torch.testing.assert_close(res[0][1], res[1][1])  # same rows seen from both ranks


def test_dlrm_single_process():
    from ps_amd.models.dlrm import DLRM, dlrm_batch

    m = DLRM(dense_in=13, table_rows=[100] * 3, dim=8, bottom=(16,), top=(16,))
    dense, sparse, y = dlrm_batch(32, [100] * 3)
    out = m(dense, sparse)
    assert out.shape == (32,)
    F.binary_cross_entropy_with_logits(out, y).backward()
    assert m.push_sparse() > 0

"""North-star configs on one MI355X (small shapes): every path runs through the HIP kernels
(fused Adam / Adagrad / row-wise sparse Adagrad / lazy-init gather / segment reduce)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def test_bert_small_ssp_gpu():
    from ps_amd.models.transformer import BertConfig, BertForMLM, mlm_batch
    from ps_amd.parallel.colocated import ColocatedPS
    from ps_amd.parallel.updaters import AdamUpdater

    torch.manual_seed(0)
    m = BertForMLM(BertConfig(vocab=1000, hidden=128, layers=2, heads=4, ffn=256, max_pos=64, dropout=0.0))
    m = m.cuda().to(torch.bfloat16)
    ps = ColocatedPS(m, AdamUpdater(2e-3, bias_correction="step"), staleness=1, bucket_mb=0.5)
    ids, labels = mlm_batch(32, 32, vocab=1000, device="cuda")
    losses = []
    for _ in range(25):
        loss = m(ids, labels)
        loss.backward()
        ps.finish_step()
        losses.append(loss.item())
    assert losses[-1] < losses[0] - 1.0


def test_dlrm_gpu_sparse_adagrad():
    from ps_amd.models.dlrm import DLRM, dlrm_batch
    from ps_amd.parallel.colocated import ColocatedPS
    from ps_amd.parallel.updaters import AdagradUpdater

    torch.manual_seed(0)
    rows = [10000] * 8
    m = DLRM(table_rows=rows, dim=64, bottom=(128,), top=(128, 64), device="cuda").cuda()
    ps = ColocatedPS(m, AdagradUpdater(0.05, 1e-8), bucket_mb=1)
    dense, sparse, y = dlrm_batch(2048, rows, device="cuda")
    before = m.emb.table.table.clone()
    losses = []
    for _ in range(15):
        loss = F.binary_cross_entropy_with_logits(m(dense, sparse), y)
        loss.backward()
        m.push_sparse()
        ps.finish_step()
        losses.append(loss.item())
    assert losses[-1] < losses[0]
    touched = m.emb.table.flags.nonzero().flatten()
    assert touched.numel() > 0
    assert (m.emb.table.table[touched] != before[touched]).any()


def test_llama_tiny_gpu():
    from ps_amd.models.transformer import LlamaConfig, LlamaForCausalLM
    from ps_amd.parallel.colocated import ColocatedPS
    from ps_amd.parallel.updaters import AdamUpdater

    torch.manual_seed(0)
    m = LlamaForCausalLM(LlamaConfig.tiny(), checkpointing=True).cuda().to(torch.bfloat16)
    ps = ColocatedPS(m, AdamUpdater(3e-3, bias_correction="step"), bucket_mb=0.5)
    ids = torch.randint(0, 512, (8, 64), device="cuda")
    losses = []
    for _ in range(15):
        loss = m(ids, ids)
        loss.backward()
        ps.finish_step()
        losses.append(loss.item())
    assert losses[-1] < losses[0]


def test_reference_models_gpu():
    from ps_amd.context import ctx
    from ps_amd.data.dataset import synthetic_ctr
    from ps_amd.models.reference import CNN, DNN, WideDeepNN, local_table_factory
    from ps_amd.train.trainer import CollectiveEngine, Trainer

    ctx.init()
    dev = torch.device("cuda")
    m = WideDeepNN.build_model(5, 4, 6, [16, 8, 1], 1000, gen=torch.Generator().manual_seed(0), emb_rows=4096,
                               init_scale=0.1, table_factory=local_table_factory(device=dev)).to(dev)
    tr = Trainer(m, CollectiveEngine(m), device=dev)
    losses = [tr.train([synthetic_ctr(256, fields=5, numeric=6, ids_per_field=50, wide_k=5, wide_size=1000,
                                      seed=i)]) for i in range(20)]
    assert losses[-1] < losses[0]
    c = CNN.build_model(28, 28, 1, [150, 50, 10], gen=torch.Generator().manual_seed(0)).to(dev)
    tr2 = Trainer(c, CollectiveEngine(c), device=dev)
    x = torch.rand(64, 784)
    y = torch.randint(0, 10, (64,))
    l0 = tr2.train([{"X": x, "Y": y}])
    for _ in range(10):
        l1 = tr2.train([{"X": x, "Y": y}])
    assert l1 < l0

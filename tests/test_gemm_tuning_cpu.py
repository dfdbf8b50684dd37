"""ps_amd/utils/gemm_tuning.py: the tuned-GEMM table loader is a no-op unless a table exists, the
device is a gfx950 GPU, and PS_AMD_GEMM_TUNING allows it (profiles/r5_llama_tunableop_ab.txt)."""
import torch

from ps_amd.utils import gemm_tuning


def test_no_table_means_no_tunableop(monkeypatch, tmp_path):
    monkeypatch.setenv("PS_AMD_GEMM_TUNING", "auto")
    assert gemm_tuning.table_for("no-such-config") is None
    monkeypatch.setenv("PS_AMD_GEMM_TUNING", "off")
    assert gemm_tuning.table_for("llama-onebit") is None
    t = tmp_path / "t.csv"
    t.write_text("Validator,PT_VERSION,0\n")
    monkeypatch.setenv("PS_AMD_GEMM_TUNING", str(t))
    assert gemm_tuning.table_for("llama-onebit") == str(t)
    # CPU device: never touches TunableOp
    assert gemm_tuning.load("llama-onebit", torch.device("cpu")) is None

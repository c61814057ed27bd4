"""FeatureResult.csr() compaction (ops/text.py): rows written at arbitrary slot bases (with
empty rows and gaps) are gathered into CSR order exactly like the per-entry row-index formula."""
import pytest
import torch

from fraud_detection_spark_kafka_llm_amd.ops.text import FeatureResult


@pytest.mark.parametrize("dev", ["cpu", pytest.param("cuda:0", marks=pytest.mark.gpu)])
def test_compaction_equals_row_index_gather(dev):
    g = torch.Generator().manual_seed(0)
    for trial in range(60):
        D = int(torch.randint(1, 300, (1,), generator=g))
        nnz = torch.randint(0, 9, (D,), generator=g).to(torch.int32)
        if trial % 7 == 0:
            nnz[:] = 0
        if trial % 5 == 0:
            nnz[0] = 0
        base = torch.zeros(D, dtype=torch.int64)
        pos = 0
        for r in torch.randperm(D, generator=g).tolist():      # shuffled slots with gaps
            pos += int(torch.randint(0, 3, (1,), generator=g))
            base[r] = pos
            pos += int(nnz[r])
        idx = torch.randint(0, 1 << 18, (pos + 2,), generator=g).to(torch.int32)
        val = torch.rand(pos + 2, generator=g)
        fr = FeatureResult(nnz.to(dev), None, None, None, idx.to(dev), val.to(dev), base.to(dev), 1 << 18)
        ip, ix, v = fr.csr()
        n64 = nnz.to(torch.int64)
        total = int(n64.sum())
        row = torch.repeat_interleave(torch.arange(D), n64, output_size=total)
        ref_ip = torch.zeros(D + 1, dtype=torch.int64)
        torch.cumsum(n64, 0, out=ref_ip[1:])
        p = base[row] + (torch.arange(total) - ref_ip[row])
        assert torch.equal(ip.cpu(), ref_ip)
        assert torch.equal(ix.cpu(), idx[p]) and torch.equal(v.cpu(), val[p]), trial

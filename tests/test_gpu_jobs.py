"""GPU runs of the CLI job layer and the K18 GSP join kernel against their CPU oracles."""
import json
from pathlib import Path

import pytest
import torch

from avenir_amd.cli import main

FIX = Path(__file__).parent / "fixtures"


def run(dev, *args):
    assert main([str(a) for a in args] + ["--device", dev]) == 0


def lines(p):
    p = Path(p)
    if p.is_dir():
        return [l for f in sorted(p.iterdir()) if f.is_file() for l in f.read_text().splitlines() if l.strip()]
    return [l for l in p.read_text().splitlines() if l.strip()]


@pytest.mark.gpu
@pytest.mark.parametrize("k,V,N", [(2, 5, 20), (3, 6, 500), (4, 3, 81), (5, 4, 3000)])
def test_gsp_join_kernel_matches_oracle(cuda, k, V, N):
    from avenir_amd.ops import sequence_ops as SO
    g = torch.Generator().manual_seed(k * 100 + V)
    X = torch.randint(0, V, (N, k), generator=g, dtype=torch.int32)
    ref = SO.gsp_join(X)
    got = SO.gsp_join(X.to(cuda))
    torch.cuda.synchronize()
    assert torch.equal(got.cpu(), ref)
    # sub-range of left rows (the distributed path)
    U = torch.unique(X, dim=0)
    lo, hi = U.shape[0] // 3, 2 * U.shape[0] // 3
    assert torch.equal(SO.gsp_join(X.to(cuda), lo, hi).cpu(), SO.gsp_join(X, lo, hi))


@pytest.mark.gpu
def test_gsp_join_empty_and_no_partner(cuda):
    from avenir_amd.ops import sequence_ops as SO
    X = torch.tensor([[0, 1], [2, 3]], dtype=torch.int32)
    assert SO.gsp_join(X.to(cuda)).shape == (0, 3)
    X = torch.tensor([[0, 1], [1, 2]], dtype=torch.int32)
    assert SO.gsp_join(X.to(cuda)).cpu().tolist() == [[0, 1, 2]]


@pytest.mark.gpu
def test_jobs_gpu_equal_cpu(cuda, tmp_path):
    """Counting jobs give identical lines on the device path and the CPU oracle path."""
    from avenir_amd.data import synth
    data, schema = tmp_path / "churn.csv", tmp_path / "churn.json"
    synth.write_churn(data, 5000, seed=3, schema_path=schema)
    sj = json.loads(schema.read_text())
    ords = [f["ordinal"] for f in sj["fields"] if f.get("feature") and f.get("dataType") == "categorical"][:3]
    props = tmp_path / "p.properties"
    props.write_text(f"crc.feature.schema.file.path={schema}\ncrc.source.attributes={ords[0]}\n"
                     f"crc.dest.attributes={','.join(map(str, ords[1:]))}\n")
    outs = {}
    for dev in ("cpu", "cuda"):
        o = tmp_path / f"nb_{dev}.txt"
        run(dev, "bayesianDistribution", "-i", data, "-o", o, "--schema", schema)
        c = tmp_path / f"crc_{dev}.txt"
        run(dev, "cramerCorrelation", "-i", data, "-o", c, "-c", props)
        m = tmp_path / f"mi_{dev}.txt"
        run(dev, "mutualInformation", "-i", data, "-o", m, "--schema", schema)
        outs[dev] = (lines(o), lines(c), lines(m))
    assert outs["cpu"][0] == outs["cuda"][0]
    for a, b in zip(outs["cpu"][1], outs["cuda"][1]):
        assert a.rsplit(",", 1)[0] == b.rsplit(",", 1)[0]
        assert float(a.rsplit(",", 1)[1]) == pytest.approx(float(b.rsplit(",", 1)[1]), rel=1e-9)
    assert outs["cpu"][2][0] == outs["cuda"][2][0]


@pytest.mark.gpu
def test_sequence_jobs_gpu(cuda, tmp_path):
    seqs = tmp_path / "k3.txt"
    g = torch.Generator().manual_seed(5)
    X = torch.randint(0, 6, (300, 3), generator=g)
    seqs.write_text("\n".join(",".join(f"t{v}" for v in r) for r in X.tolist()))
    props = tmp_path / "c.properties"
    props.write_text("cgs.item.set.length=3\npstg.max.seq.length=3\n")
    res = {}
    for dev in ("cpu", "cuda"):
        o = tmp_path / f"cgs_{dev}.txt"
        run(dev, "candidateGenerationWithSelfJoin", "-i", seqs, "-o", o, "-c", props)
        p = tmp_path / f"pst_{dev}.txt"
        run(dev, "probabilisticSuffixTreeGenerator", "-i", seqs, "-o", p, "-c", props)
        res[dev] = (lines(o), lines(p))
    assert res["cpu"] == res["cuda"]

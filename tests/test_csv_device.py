"""K1 on the device (csrc/kernels/csv.hip): the GPU CSV parse gives exactly the host parser's
columns — dictionary codes, bucket codes, floats — including blank lines, CRLF endings, a missing
final newline, unknown values, short rows, a header and row shards."""
import os

import pytest
import torch

from avenir_amd.data import synth
from avenir_amd.data import table as TB
from avenir_amd.utils.schema import FeatureSchema


def _compare(path, schema, **kw):
    cpu = TB.load_csv(path, schema, **kw)
    gpu = TB.load_csv(path, schema, device="cuda", **kw)
    assert gpu.codes.is_cuda and gpu.n == cpu.n and gpu.row_offset == cpu.row_offset
    assert torch.equal(gpu.codes.cpu()[:, : cpu.n], cpu.codes[:, : cpu.n])
    if cpu.labels is not None:
        assert torch.equal(gpu.labels.cpu()[: cpu.n], cpu.labels[: cpu.n])
    a, b = gpu.numeric.cpu()[:, : cpu.n], cpu.numeric[:, : cpu.n]
    assert torch.equal(torch.isnan(a), torch.isnan(b)) and torch.equal(a.nan_to_num(), b.nan_to_num())
    if cpu.ids is not None:
        assert list(gpu.ids[:5]) == list(cpu.ids[:5])
    return cpu, gpu


@pytest.mark.gpu
@pytest.mark.parametrize("world", [1, 3])
def test_device_csv_matches_host_churn(cuda, tmp_path, monkeypatch, world):
    monkeypatch.setattr(TB, "_GPU_CSV_MIN_BYTES", 0)
    p = tmp_path / "churn.csv"
    synth.write_churn_native(p, 200_003, seed=4)
    schema = FeatureSchema.from_json(synth.CHURN_SCHEMA)
    for rank in range(world):
        _compare(p, schema, rank=rank, world=world)


@pytest.mark.gpu
def test_device_csv_edge_cases(cuda, tmp_path, monkeypatch):
    monkeypatch.setattr(TB, "_GPU_CSV_MIN_BYTES", 0)
    lines = synth.call_hangup_lines(5000, seed=3)
    lines[7] = lines[7].replace("business", "unknownType")          # unknown dictionary value
    lines[9] = ",".join(lines[9].split(",")[:3])                     # short row
    lines[11] = lines[11].replace(",", " , ")                       # padded fields (trimmed)
    body = "\r\n".join(lines[:100]) + "\r\n\r\n" + "\n".join(lines[100:]) + "\n\n"
    p = tmp_path / "h.csv"
    p.write_text("id,a,b,c,d,e,f\n" + body.rstrip("\n"))              # header, no final newline
    schema = FeatureSchema.from_json(synth.CALL_HANGUP_SCHEMA)
    _compare(p, schema, skip_header=True)
    _compare(p, schema, skip_header=True, raw_numeric=True)

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


def _wide_file(path, n_rows, n_cols=80, seed=0):
    """``id,c1..c{n_cols-1},class``: categorical / bucketed int / float columns in turn."""
    import numpy as np
    rng = np.random.default_rng(seed)
    cols = [np.char.add("r", np.arange(n_rows).astype(str))]
    fields = [{"name": "id", "ordinal": 0, "id": True, "dataType": "string"}]
    for j in range(1, n_cols):
        k = j % 3
        if k == 0:
            cols.append(np.array(["aa", "bb", "cc", "dd"])[rng.integers(0, 4, n_rows)])
            fields.append({"name": f"c{j}", "ordinal": j, "dataType": "categorical", "feature": True,
                           "cardinality": ["aa", "bb", "cc", "dd"]})
        elif k == 1:
            cols.append(rng.integers(0, 100, n_rows).astype(str))
            fields.append({"name": f"c{j}", "ordinal": j, "dataType": "int", "feature": True, "bucketWidth": 10,
                           "min": 0, "max": 99})
        else:
            cols.append(np.char.mod("%.3f", rng.normal(size=n_rows)))
            fields.append({"name": f"c{j}", "ordinal": j, "dataType": "double", "feature": True})
    cols.append(np.array(["T", "F"])[rng.integers(0, 2, n_rows)])
    fields.append({"name": "cls", "ordinal": n_cols, "dataType": "categorical", "classAttribute": True,
                   "cardinality": ["T", "F"]})
    with open(path, "w") as f:
        for a in range(0, n_rows, 20000):
            rows = [",".join(c[i] for c in cols) for i in range(a, min(n_rows, a + 20000))]
            f.write("\n".join(rows) + "\n")
    return FeatureSchema.from_json({"fields": fields})


def test_wide_schema_host_parse_keeps_line_spans(tmp_path):
    """The host parser on an 80-column schema; lines kept as byte spans equal the file's lines."""
    p = tmp_path / "wide.csv"
    schema = _wide_file(p, 3000)
    t = TB.load_csv(p, schema, keep_lines=True)
    assert t.n == 3000 and t.meta["parser"] == "host" and len(t.binned_fields) > 32
    assert t.lines.tolist() == p.read_text().splitlines()
    sub = t.select_rows(torch.tensor([5, 2, 2999]))
    assert list(sub.lines) == [p.read_text().splitlines()[i] for i in (5, 2, 2999)]


@pytest.mark.gpu
def test_device_csv_wide_schema_over_32mb(cuda, tmp_path):
    """> 32 parsed columns used to throw inside csv_parse_device.  80 columns, a file
    above the 32 MB device threshold: the device parse (passes of <= 64 columns) equals the host
    parse, reports parser='device', and its line spans equal the host lines."""
    p = tmp_path / "wide.csv"
    schema = _wide_file(p, 110_000)
    assert os.path.getsize(p) >= TB._GPU_CSV_MIN_BYTES
    cpu, gpu = _compare(p, schema, keep_lines=True)
    assert gpu.meta.get("parser") == "device"
    assert gpu.codes.shape[0] + gpu.numeric.shape[0] >= 79
    assert gpu.lines[:100].tolist() == cpu.lines[:100].tolist()
    assert gpu.lines[-3:].tolist() == cpu.lines[-3:].tolist() and len(gpu.lines) == len(cpu.lines)


@pytest.mark.gpu
def test_device_csv_full_precision_doubles(cuda, tmp_path, monkeypatch):
    """the device CSV parser rounds full-precision doubles (repr / Java Double.toString,
    subnormals, long exponents: the Eisel-Lemire tier of avenir_numparse.h) exactly as the host
    parser, so the column bits do not depend on which parser the file size picks; a token the
    device cannot settle (> 19 digits on a rounding midpoint) sends the file to the host parser."""
    import random
    import struct
    monkeypatch.setattr(TB, "_GPU_CSV_MIN_BYTES", 0)
    rnd = random.Random(11)
    vals = []
    while len(vals) < 20000:
        d = struct.unpack("<d", struct.pack("<Q", rnd.getrandbits(64)))[0]
        if d == d and abs(d) < 1e300:
            vals.append(repr(d))
    vals += [repr(rnd.uniform(1, 10) * 10.0 ** -rnd.randint(300, 323)) for _ in range(500)]
    fields = [{"name": "id", "ordinal": 0, "id": True, "dataType": "string"},
              {"name": "x", "ordinal": 1, "dataType": "double", "feature": True},
              {"name": "cls", "ordinal": 2, "dataType": "categorical", "classAttribute": True,
               "cardinality": ["T", "F"]}]
    schema = FeatureSchema.from_json({"fields": fields})
    p = tmp_path / "dbl.csv"
    p.write_text("".join(f"r{i},{v},{'TF'[i % 2]}\n" for i, v in enumerate(vals)))
    for raw in (False, True):
        cpu, gpu = _compare(p, schema, raw_numeric=raw)
    p2 = tmp_path / "amb.csv"
    p2.write_text("".join(f"r{i},{'9007199254740993.0000000000001' if i == 5 else v},{'TF'[i % 2]}\n"
                          for i, v in enumerate(vals[:3000])))
    _compare(p2, schema, raw_numeric=True)

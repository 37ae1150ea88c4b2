"""Native record ingest (data/records.py, csrc/host/records.cpp, csrc/kernels/records.hip).

CPU: the native TextShard tokenizer against its pure-Python twin, byte-range shards at several
world sizes (every line on exactly one rank; merged dictionaries = world-1 dictionary), and the
JobContext line shards.  GPU: the device tokenizer against the host tokenizer (codes, sub codes,
numbers, vocabulary), sharded and whole."""
from __future__ import annotations

import math
import random

import pytest
import torch

from avenir_amd import _native
from avenir_amd.data import records as R

from _dist import run_world


def _write(tmp_path, n=3000, seed=0, crlf=True, name="rec.txt"):
    rnd = random.Random(seed)
    st = ["L", "M", "H", "LL", "hm", "x y"]
    lines = []
    for i in range(n):
        toks = [f"{rnd.choice(st)}:{rnd.choice('abc')}" for _ in range(rnd.randint(1, 9))]
        lines.append(f"id{i},{rnd.random() * 100:.3f}," + ",".join(toks))
        if i % 97 == 0:
            lines.append("  \t ")
    txt = "".join(l + ("\r\n" if crlf and i % 3 == 0 else "\n") for i, l in enumerate(lines))
    p = tmp_path / name
    p.write_text(txt.rstrip("\n"))   # last line without a newline
    return p


SPECS = [dict(), dict(sub_delim=":"), dict(modes="xn", numeric=True), dict(modes="dn", sub_delim=":", numeric=True,
                                                                              trim=True)]


def _py(paths, rank=0, world=1, **kw):
    return R._read_records_py(paths, rank, world, kw.get("delims", ","), kw.get("sub_delim", ""), kw.get("modes", ""),
                              kw.get("tail_mode", "d"), kw.get("trim", False), kw.get("numeric", False), False)


def _same(a, b):
    assert a.vocab == b.vocab
    assert torch.equal(a.off.cpu(), b.off.cpu())
    assert torch.equal(a.codes.cpu(), b.codes.cpu())
    assert (a.sub is None) == (b.sub is None)
    if a.sub is not None:
        assert torch.equal(a.sub.cpu(), b.sub.cpu())
    if a.nums is not None:
        assert torch.allclose(a.nums.cpu(), b.nums.cpu(), equal_nan=True)


@pytest.mark.skipif(not _native.available(), reason="native extension not built")
@pytest.mark.parametrize("spec", SPECS)
def test_native_tokenizer_matches_python(tmp_path, spec):
    p = _write(tmp_path)
    _same(R.read_records(str(p), **spec), _py([str(p)], **spec))


@pytest.mark.skipif(not _native.available(), reason="native extension not built")
@pytest.mark.parametrize("world", [2, 3, 8])
def test_byte_range_shards_partition_lines(tmp_path, world):
    a = _write(tmp_path, n=2000, seed=1, name="part-00000")
    _write(tmp_path, n=1500, seed=2, name="part-00001")
    whole = R.shard_lines(str(tmp_path))
    C = _native.C()
    parts, bytes_read = [], 0
    for r in range(world):
        sh = C.TextShard([str(tmp_path / "part-00000"), str(tmp_path / "part-00001")], r, world, 4, False)
        parts += sh.lines(0, sh.num_lines())
        bytes_read += sh.bytes_read()
        # the python twin makes the same ownership decision
        assert sh.lines(0, sh.num_lines()) == R._py_lines([str(tmp_path / "part-00000"),
                                                           str(tmp_path / "part-00001")], r, world, False)
    assert parts == whole
    # every byte is read by exactly one rank (plus nothing else)
    assert bytes_read == a.stat().st_size + (tmp_path / "part-00001").stat().st_size


def _rank_records(rank, world, path):
    from avenir_amd.parallel.comm import get_comm
    rec = R.read_records(path, comm=get_comm(), sub_delim=":", modes="xn", numeric=True)
    return rec.line_base, rec.n_lines, rec.vocab, rec.codes.tolist(), rec.sub.tolist()


@pytest.mark.skipif(not _native.available(), reason="native extension not built")
def test_merged_dictionary_is_world_invariant(tmp_path):
    p = _write(tmp_path, n=4000, seed=3)
    one = R.read_records(str(p), sub_delim=":", modes="xn", numeric=True)
    res = run_world(_rank_records, 4, str(p))
    codes, subs, base = [], [], 0
    for lb, n, voc, c, s in res:
        assert voc == one.vocab          # the merged dictionary is the world-1 dictionary
        assert lb == base
        base += n
        codes += c
        subs += s
    assert base == one.n_lines
    assert codes == one.codes.tolist() and subs == one.sub.tolist()


def test_records_helpers(tmp_path):
    p = tmp_path / "f.txt"
    p.write_text("a,1.5,x\nb,2,y,z\n\nc,bad,x\n")
    rec = R.read_records(str(p), modes="dn", numeric=True)
    assert rec.n_lines == 3 and rec.width() is None
    assert rec.strings(rec.field(0)) == ["a", "b", "c"]
    f1 = rec.field(1, numeric=True)
    assert f1[0] == 1.5 and f1[1] == 2 and math.isnan(float(f1[2]))
    assert rec.strings(rec.field(-1)) == ["x", "z", "x"]
    assert rec.field(3).tolist() == [-1, rec.vocab.index("z"), -1]
    assert rec.map_codes(rec.field(0), ["c", "a"]).tolist() == [1, -1, 0]


@pytest.mark.gpu
@pytest.mark.parametrize("spec", SPECS)
@pytest.mark.parametrize("world", [1, 3])
def test_device_tokenizer_matches_host(tmp_path, cuda, spec, world):
    p = _write(tmp_path, n=20000, seed=4)
    C = _native.C()
    for r in range(world):
        out = C.text_tokenize_device([str(p)], r, world, ",", spec.get("sub_delim", ""), spec.get("modes", ""), "d",
                                     spec.get("trim", False), spec.get("numeric", False), torch.empty(0, device=cuda))
        assert out is not None
        off, codes, sub, nums, vocab, stats = out
        assert codes.is_cuda and off.is_cuda
        sh = C.TextShard([str(p)], r, world, 4, False)
        hoff, hcodes, hsub, hnums, hvocab = sh.tokenize(",", spec.get("sub_delim", ""), spec.get("modes", ""), "d",
                                                        spec.get("trim", False), spec.get("numeric", False))
        _same(R.Records(off, codes, sub, nums, list(vocab)), R.Records(hoff, hcodes, hsub, hnums, list(hvocab)))


@pytest.mark.gpu
def test_device_tokenizer_large_vocab_and_table_growth(tmp_path, cuda, monkeypatch):
    # 300k distinct ids + a small vocabulary; a 1024-slot first table forces the retry path
    p = tmp_path / "ids.txt"
    rnd = random.Random(5)
    p.write_text("\n".join(f"u{i * 7919 % 1000003},{rnd.choice('ABCD')},{i % 13}" for i in range(300_000)) + "\n")
    monkeypatch.setattr(R, "DEVICE_MIN_BYTES", 0)
    dev = R.read_records(str(p), device=cuda, modes="ddn", numeric=True)
    assert dev.stats.get("path") == "device"
    host = R.read_records(str(p), modes="ddn", numeric=True)
    _same(dev, host)
    off, codes, sub, nums, vocab, stats = _native.C().text_tokenize_device(
        [str(p)], 0, 1, ",", "", "ddn", "d", False, True, torch.empty(0, device=cuda), 1024)
    assert stats["table_slots"] >= 2 * len(host.vocab)
    _same(R.Records(off, codes, sub, nums, list(vocab)), host)


@pytest.mark.gpu
def test_device_csv_ring_two_threads(tmp_path, cuda):
    """concurrent device CSV loads must not share staging slots."""
    import threading
    from avenir_amd.data import table as T
    from avenir_amd.data.table import load_csv
    from avenir_amd.utils.schema import FeatureSchema
    schema = FeatureSchema.from_json({"fields": [
        {"name": "id", "ordinal": 0, "dataType": "string", "id": True},
        {"name": "a", "ordinal": 1, "dataType": "categorical", "feature": True, "cardinality": ["x", "y", "z"]},
        {"name": "c", "ordinal": 2, "dataType": "categorical", "cardinality": ["0", "1"]}]})
    paths = []
    for k in range(2):
        p = tmp_path / f"t{k}.csv"
        rnd = random.Random(k)
        p.write_text("\n".join(f"r{i},{rnd.choice('xyz')},{rnd.randint(0, 1)}" for i in range(400_000)) + "\n")
        paths.append(p)
    old = T._GPU_CSV_MIN_BYTES
    T._GPU_CSV_MIN_BYTES = 1
    try:
        res = [None, None]

        def load(k):
            res[k] = load_csv(str(paths[k]), schema, ",", device=cuda)

        th = [threading.Thread(target=load, args=(k,)) for k in range(2)]
        for t in th:
            t.start()
        for t in th:
            t.join()
    finally:
        T._GPU_CSV_MIN_BYTES = old
    for k in range(2):
        ref = load_csv(str(paths[k]), schema, ",")
        assert torch.equal(res[k].codes[:, : ref.n].cpu(), ref.codes[:, : ref.n])
        assert torch.equal(res[k].labels[: ref.n].cpu(), ref.labels[: ref.n])


@pytest.mark.gpu
def test_col_moments_empty_matches_cpu(cuda):
    """an empty column behaves the same on both devices."""
    from avenir_amd.ops import encode_ops as E
    x = torch.zeros(2, 0)
    a = E.column_moments(x)
    b = E.column_moments(x.to(cuda)).cpu()
    assert torch.equal(a[:, 0], b[:, 0])
    assert torch.allclose(a, b, equal_nan=True)
    y = torch.full((1, 100), float("nan"))
    assert torch.allclose(E.column_moments(y), E.column_moments(y.to(cuda)).cpu(), equal_nan=True)


@pytest.mark.parametrize("dev", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
def test_sorted_keys_string_order(tmp_path, dev, monkeypatch):
    """Reducer key order = Python string order, from packed byte keys (device gather when the
    device tokenizer kept the dictionary bytes), including multi-byte UTF-8 and > 21-byte keys."""
    rnd = random.Random(9)
    alpha = "aAbZ09_é€"
    keys = {"".join(rnd.choice(alpha) for _ in range(rnd.randint(0, 8))) for _ in range(3000)}
    keys |= {"k" * 20, "k" * 21, "k" * 20 + "a"}
    p = tmp_path / "k.txt"
    p.write_text("\n".join(f"{k},x" for k in sorted(keys, key=lambda _: rnd.random())) + "\n", encoding="utf-8")
    monkeypatch.setattr(R, "DEVICE_MIN_BYTES", 0)
    rec = R.read_records(str(p), device=dev, modes="dx")
    ks, pos = R.sorted_keys(rec, rec.field(0))
    got = rec.strings(ks)
    assert got == sorted(k for k in keys if k)  or got == sorted(keys)
    short = {k for k in keys if len(k.encode()) <= 21}
    p2 = tmp_path / "k2.txt"
    p2.write_text("\n".join(f"{k},x" for k in short) + "\n", encoding="utf-8")
    rec2 = R.read_records(str(p2), device=dev, modes="dx")
    ks2, _ = R.sorted_keys(rec2, rec2.field(0))
    assert rec2.strings(ks2) == sorted(short)


_NUM_TOKENS = ["0.3", "0.1", "-0.7", "123.456", "1e-5", "2.5E+3", "000.0625", ".5", "5.", "9007199254740993",
               "0.30000000000000004", "1.7976931348623157e308", "4.9e-324", "123456789012345678901234.5",
               "3.141592653589793238", "1e", "--1", "1.2.3", "", " 42 ", "7e22", "1e23", "0.000000000000000000001"]


def _num_file(tmp_path, reps=1):
    p = tmp_path / "nums.txt"
    p.write_text("".join(f"r{i},{t}\n" for i in range(reps) for t in _NUM_TOKENS))
    return p


def _py_float(t):
    try:
        v = float(t.strip(" \t\r\v\f"))
    except ValueError:
        return math.nan
    return v if t.strip()[-1:].isdigit() or t.strip().endswith(".") else math.nan


@pytest.mark.skipif(not _native.available(), reason="native extension not built")
def test_numeric_tokens_are_correctly_rounded(tmp_path):
    """the native decimal parser rounded on every fractional digit ("0.3" ->
    0.30000000000000004).  Native host tokens now equal Python's float() bit for bit (and the
    pure-Python twin), including the strtod fallback beyond the exact fast path."""
    p = _num_file(tmp_path)
    nat = R.read_records(str(p), modes="xn", numeric=True).field(1, numeric=True).tolist()
    py = _py(str(p) and [str(p)], modes="xn", numeric=True).field(1, numeric=True).tolist()
    want = [_py_float(t) for t in _NUM_TOKENS]
    for t, a, b, w in zip(_NUM_TOKENS, nat, py, want):
        if math.isnan(w):
            assert math.isnan(a), t
            continue
        assert a == w and b == w, (t, a, b, w)


def _hard_tokens(n=3000, seed=5):
    """Full-precision doubles (repr: up to 17 digits, any exponent), subnormals, 18-19 digit
    mantissas and long exponents: the Eisel-Lemire tier of avenir_numparse.h."""
    import random as _r
    import struct
    rnd = _r.Random(seed)
    out = []
    while len(out) < n:
        d = struct.unpack("<d", struct.pack("<Q", rnd.getrandbits(64)))[0]
        if math.isfinite(d):
            out.append(repr(d))
    out += [repr(rnd.uniform(1, 10) * 10.0 ** -rnd.randint(300, 323)) for _ in range(300)]        # subnormals
    out += [f"{rnd.randint(10**17, 10**19 - 1)}e{rnd.randint(-330, 290)}" for _ in range(300)]      # 18-19 digits
    out += ["2.4703282292062328e-324", "2.2250738585072011e-308", "1.7976931348623158e308", "9007199254740993"]
    return out


@pytest.mark.skipif(not _native.available(), reason="native extension not built")
def test_host_parser_correctly_rounds_full_precision_doubles(tmp_path):
    toks = _hard_tokens()
    p = tmp_path / "hard.txt"
    p.write_text("".join(f"r{i},{t}\n" for i, t in enumerate(toks)))
    nat = R.read_records(str(p), modes="xn", numeric=True).field(1, numeric=True).tolist()
    assert nat == [float(t) for t in toks]


@pytest.mark.gpu
def test_device_numeric_tokens_match_host(tmp_path, cuda, monkeypatch):
    """The device tokenizer shares the parser: identical bits for EVERY token — the
    Clinger fast path, full-precision doubles, subnormals and > 19-digit mantissas through
    Eisel-Lemire — and equal to Python's float()."""
    toks = _NUM_TOKENS * 50 + _hard_tokens()
    p = tmp_path / "nums.txt"
    p.write_text("".join(f"r{i},{t}\n" for i, t in enumerate(toks)))
    monkeypatch.setattr(R, "DEVICE_MIN_BYTES", 0)
    dev = R.read_records(str(p), device=cuda, modes="xn", numeric=True)
    assert dev.stats.get("path") == "device"
    host = R.read_records(str(p), modes="xn", numeric=True)
    a, b = dev.field(1, numeric=True).cpu(), host.field(1, numeric=True)
    assert torch.equal(torch.isnan(a), torch.isnan(b))
    ok = ~torch.isnan(b)
    assert torch.equal(a[ok], b[ok])
    want = torch.tensor([_py_float(t) for t in toks], dtype=torch.float64)
    assert torch.equal(a[ok], want[ok])


@pytest.mark.gpu
def test_device_tokenizer_hands_undecidable_numbers_to_the_host(tmp_path, cuda, monkeypatch):
    """A 29-digit token a hair above the midpoint 2^53 + 1: its first 19 digits alone sit exactly on
    the midpoint (round to even -> 2^53), so the device cannot settle it; the shard goes to the
    host tokenizer (strtod), which rounds up to 2^53 + 2 like Python's float()."""
    tok = "9007199254740993.0000000000001"
    p = tmp_path / "amb.txt"
    p.write_text("".join(f"r{i},{tok if i == 777 else '1.5'}\n" for i in range(2000)))
    monkeypatch.setattr(R, "DEVICE_MIN_BYTES", 0)
    rec = R.read_records(str(p), device=cuda, modes="xn", numeric=True)
    assert rec.stats.get("path") == "host"
    assert rec.field(1, numeric=True)[777].item() == float(tok) == 9007199254740994.0


def test_format_lines_pyrepr_and_raw_kinds(tmp_path):
    """``prec=-2`` is Python's repr (shortest round trip); ``r`` / ``rf`` / ``rt`` copy raw line
    bytes (whole, one field, fields from one on) — native and pure-Python formatter agree."""
    import random as _r
    from avenir_amd.data.lines import LineSpans
    rnd = _r.Random(1)
    v = torch.tensor([0.1 + 0.2, -0.0, 1e16, 1.5e-5, 123.0, 1e-4, 5e-324, float("inf"), float("nan")]
                     + [rnd.uniform(-1, 1) * 10 ** rnd.randint(-25, 25) for _ in range(500)], dtype=torch.float64)
    got = R.format_lines([("f", v, -2)], v.numel()).decode().split()
    assert got == [repr(x) for x in v.tolist()]
    p = tmp_path / "l.txt"
    p.write_text("a,b,c\nd|e,f\n\ng\n")
    sh = _native.C().TextShard([str(p)], 0, 1, 2, False) if _native.available() else None
    spans = LineSpans.from_shard(sh) if sh is not None else LineSpans.from_strings(["a,b,c", "d|e,f", "g"])
    assert spans.tolist() == ["a,b,c", "d|e,f", "g"] and spans[1] == "d|e,f" and len(spans) == 3
    cols = [spans.column("rf", 1, ",|"), spans.column("rf", -1, ","), spans.column("rt", 1, ",|"),
            spans.column("r", delims=",")]
    want = "b;c;b;c;a;b;c\ne;f;e;f;d|e;f\n;g;;g\n"
    assert R.format_lines(cols, 3, ";").decode() == want
    C = _native.host
    try:
        _native.host = lambda: None          # the pure-Python twin
        assert R.format_lines(cols, 3, ";").decode() == want
    finally:
        _native.host = C

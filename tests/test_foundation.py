"""Config / schema / CSV (K1) / metrics foundation tests (CPU)."""
import json
import math

import pytest
import torch

from avenir_amd.data import synth
from avenir_amd.data.table import load_csv, shard_range
from avenir_amd.utils.config import Configuration, JobConfig, parse_hocon, parse_properties
from avenir_amd.utils.schema import FeatureSchema


def test_properties_parsing():
    p = parse_properties("# c\nfield.delim.regex=,\na.b : x y\nc\\\n  d=1\n! bang\nkey\\=x=5\n")
    assert p["field.delim.regex"] == ","
    assert p["a.b"] == "x y"
    assert p["cd"] == "1"
    assert p["key=x"] == "5"


def test_hocon_blocks():
    h = parse_hocon('app {\n a.b = 3\n s = "x y" // c\n arr = ["1:2", "3"]\n sub { k = true }\n}\n')
    assert h["app"]["a.b"] == 3 and h["app"]["s"] == "x y"
    assert h["app"]["arr"] == ["1:2", "3"] and h["app"]["sub"]["k"] is True


def test_jobconfig_prefix_fallback(tmp_path):
    f = tmp_path / "x.properties"
    f.write_text("num.reducer=4\ndtb.max.depth.limit=2\nfield.delim.regex=\\\\t\n")
    c = JobConfig.from_file(f, prefix="dtb.")
    assert c.get_int("num.reducer") == 4 and c.get_int("max.depth.limit") == 2
    with pytest.raises(KeyError):
        c.get_int("missing.key")
    assert c.get_int("missing.key", 7) == 7


def test_configuration_defaults():
    c = Configuration({"a": "_", "b": "none", "c": "3"}, {"a": (5, None), "b": (1, None),
                                                           "c": (0, None), "d": (None, "d is mandatory")})
    assert c.get_int("a") == (5, True)
    assert c.get_int("b") == (None, False)
    assert c.get_int("c") == (3, False)
    with pytest.raises(ValueError):
        c.get_int("d")


def test_reference_configs_parse(ref_resource):
    JobConfig.from_file(ref_resource("opt.conf"), app="simulatedAnnealing")
    JobConfig.from_file(ref_resource("samp.conf"), app="multiArmBandit")
    JobConfig.from_file(ref_resource("detr.properties"))


def test_schema(ref_resource):
    s = FeatureSchema.from_json(ref_resource("call_hangup.json"))
    assert s.find_class_attr_field().name == "hungup"
    hold = s.find_field_by_name("hold time")
    assert hold.is_bucketed and hold.num_bins == 11
    s2 = FeatureSchema.from_json(json.loads(s.dumps()))
    assert [f.name for f in s2.fields] == [f.name for f in s.fields]


def test_csv_load_matches_python(tmp_path):
    p = tmp_path / "churn.csv"
    synth.write_churn(p, 1000, seed=3)
    schema = FeatureSchema.from_json(synth.CHURN_SCHEMA)
    t = load_csv(p, schema)
    assert t.n == 1000 and t.codes.shape == (5, 1008)
    lines = p.read_text().splitlines()
    for r in (0, 17, 999):
        it = lines[r].split(",")
        for j, f in enumerate(t.binned_fields):
            assert f.cardinality[t.codes[j, r]] == it[f.ordinal]
        assert t.class_field.cardinality[t.labels[r]] == it[6]
    assert t.ids[5] == lines[5].split(",")[0]
    # padding is the missing sentinel
    assert int(t.codes[0, 1000:].min()) == 255


def test_csv_sharding(tmp_path):
    p = tmp_path / "c.csv"
    synth.write_churn(p, 103, seed=1)
    schema = FeatureSchema.from_json(synth.CHURN_SCHEMA)
    full = load_csv(p, schema)
    parts = [load_csv(p, schema, rank=r, world=4) for r in range(4)]
    assert sum(x.n for x in parts) == 103
    cat = torch.cat([x.codes[:, : x.n] for x in parts], dim=1)
    assert torch.equal(cat, full.codes[:, :103])
    assert shard_range(10, 3, 4) == (8, 10)


def test_csv_bucketize(tmp_path, ref_resource):
    schema = FeatureSchema.from_json(ref_resource("call_hangup.json"))
    p = tmp_path / "h.csv"
    p.write_text("\n".join(synth.call_hangup_lines(200, seed=2)) + "\n")
    t = load_csv(p, schema)
    lines = p.read_text().splitlines()
    hold_idx = [f.name for f in t.binned_fields].index("hold time")
    for r in range(0, 200, 37):
        v = int(lines[r].split(",")[5])
        assert int(t.codes[hold_idx, r]) == v // 60


def test_metrics():
    from avenir_amd.utils.metrics import ConfusionMatrix, perf_metric, roc_auc
    cm = ConfusionMatrix("open", "closed")
    for p, a in [("closed", "closed"), ("closed", "open"), ("open", "open"), ("open", "closed")]:
        cm.report(p, a)
    assert (cm.tp, cm.fp, cm.tn, cm.fn) == (1, 1, 1, 1) and cm.accuracy == 50
    assert math.isclose(roc_auc([0, 0, 1, 1], [0.1, 0.4, 0.35, 0.8]), 0.75)
    assert perf_metric("acc", [1, 0, 1], [1, 1, 1]) == pytest.approx(2 / 3)


def test_schema_entity_format_with_class_attribute():
    """sifarish-style schema (resource/elearnActivity.json layout): fields under "entity", every
    non-id non-class field a feature, the class marked by "classAttribute"."""
    from avenir_amd.utils.schema import FeatureSchema
    d = {"distAlgorithm": "euclidean", "numericDiffThreshold": 0.2,
         "entity": {"name": "studentActivity", "fields": [
             {"name": "studentID", "ordinal": 0, "id": True, "dataType": "string"},
             {"name": "contentTime", "ordinal": 1, "dataType": "int", "min": 0, "max": 600},
             {"name": "emailCount", "ordinal": 2, "dataType": "int", "min": 0, "max": 20},
             {"name": "status", "ordinal": 3, "dataType": "categorical", "classAttribute": True,
              "cardinality": ["pass", "fail"]}]}}
    s = FeatureSchema.from_json(d)
    assert [f.name for f in s.feature_fields] == ["contentTime", "emailCount"]
    assert s.find_class_attr_field().name == "status"
    assert s.extra["entityName"] == "studentActivity" and s.extra["distAlgorithm"] == "euclidean"

"""JSON FeatureSchema — the reference's cross-cutting data contract, read unchanged.

Format (e.g. ``resource/churn.json``, ``resource/call_hangup.json``): ``{"fields": [ {name,
ordinal, dataType: categorical|int|double|string, id, feature, cardinality[], bucketWidth, min,
max, maxSplit, splitScanInterval, weight}, ... ]}``.  The class attribute is the field that is
neither ``id`` nor ``feature`` (chombo ``FeatureSchema.findClassAttrField()``, used at
``src/main/java/org/avenir/bayesian/BayesianDistribution.java:122``).
"""
from __future__ import annotations

import json
import math
from dataclasses import dataclass, field
from pathlib import Path
from typing import Any


@dataclass
class FeatureField:
    name: str
    ordinal: int
    data_type: str = "string"
    id: bool = False
    feature: bool = False
    cardinality: list[str] | None = None
    bucket_width: float | None = None
    min: float | None = None
    max: float | None = None
    max_split: int | None = None
    split_scan_interval: float | None = None
    weight: float = 1.0
    extra: dict[str, Any] = field(default_factory=dict)

    @classmethod
    def from_json(cls, d: dict[str, Any]) -> "FeatureField":
        known = {"name", "ordinal", "dataType", "id", "feature", "cardinality", "bucketWidth", "min",
                 "max", "maxSplit", "splitScanInterval", "weight"}
        card = d.get("cardinality")
        return cls(
            name=d.get("name", f"f{d.get('ordinal')}"),
            ordinal=int(d["ordinal"]),
            data_type=str(d.get("dataType", "string")),
            id=bool(d.get("id", False)),
            feature=bool(d.get("feature", False)),
            cardinality=[str(c) for c in card] if card is not None else None,
            bucket_width=float(d["bucketWidth"]) if d.get("bucketWidth") is not None else None,
            min=float(d["min"]) if d.get("min") is not None else None,
            max=float(d["max"]) if d.get("max") is not None else None,
            max_split=int(d["maxSplit"]) if d.get("maxSplit") is not None else None,
            split_scan_interval=(float(d["splitScanInterval"])
                                 if d.get("splitScanInterval") is not None else None),
            weight=float(d.get("weight", 1.0)),
            extra={k: v for k, v in d.items() if k not in known},
        )

    def to_json(self) -> dict[str, Any]:
        d: dict[str, Any] = {"name": self.name, "ordinal": self.ordinal, "dataType": self.data_type}
        if self.id:
            d["id"] = True
        if self.feature:
            d["feature"] = True
        if self.cardinality is not None:
            d["cardinality"] = list(self.cardinality)
        for k, v in (("bucketWidth", self.bucket_width), ("min", self.min), ("max", self.max),
                     ("maxSplit", self.max_split), ("splitScanInterval", self.split_scan_interval)):
            if v is not None:
                d[k] = int(v) if float(v).is_integer() else v
        if self.weight != 1.0:
            d["weight"] = self.weight
        d.update(self.extra)
        return d

    # -- type predicates (chombo FeatureField) -----------------------------------------------------
    @property
    def is_categorical(self) -> bool:
        return self.data_type == "categorical"

    @property
    def is_numeric(self) -> bool:
        return self.data_type in ("int", "double", "float", "long")

    @property
    def is_integer(self) -> bool:
        return self.data_type in ("int", "long")

    @property
    def is_bucketed(self) -> bool:
        return self.is_numeric and self.bucket_width is not None

    @property
    def is_binned(self) -> bool:
        """True when the field is a discrete (coded) variable: categorical or bucketized."""
        return self.is_categorical or self.is_bucketed

    @property
    def num_bins(self) -> int:
        if self.is_categorical:
            if not self.cardinality:
                raise ValueError(f"categorical field {self.name!r} has no cardinality")
            return len(self.cardinality)
        if self.is_bucketed:
            lo = self.min if self.min is not None else 0.0
            hi = self.max if self.max is not None else lo + 254 * self.bucket_width
            return max(1, int(math.floor(hi / self.bucket_width)) - self.bucket_offset + 1)
        raise ValueError(f"field {self.name!r} is not binned")

    @property
    def bucket_offset(self) -> int:
        lo = self.min if self.min is not None else 0.0
        return int(math.floor(lo / self.bucket_width)) if self.bucket_width else 0

    def bin_label(self, b: int) -> str:
        """Text of bin ``b`` in the reference's model files: the categorical value, or the
        integer bucket index ``value / bucketWidth`` (BayesianDistribution.java:150-153)."""
        if self.is_categorical:
            return self.cardinality[b]
        return str(b + self.bucket_offset)


class FeatureSchema:
    def __init__(self, fields: list[FeatureField], extra: dict[str, Any] | None = None):
        self.fields = sorted(fields, key=lambda f: f.ordinal)
        self.extra = extra or {}

    @classmethod
    def from_json(cls, obj: dict[str, Any] | str | Path) -> "FeatureSchema":
        if isinstance(obj, (str, Path)):
            p = Path(obj)
            obj = json.loads(p.read_text()) if p.exists() else json.loads(str(obj))
        if "fields" not in obj and isinstance(obj.get("entity"), dict):
            # sifarish / similarity format (e.g. resource/elearnActivity.json):
            # {"distAlgorithm": ..., "entity": {"name": ..., "fields": [...]}}; every field that is
            # neither the id nor the "classAttribute" is a feature
            ent = obj["entity"]
            fields = [FeatureField.from_json(d) for d in ent.get("fields", [])]
            for f in fields:
                if not f.id and not f.extra.get("classAttribute", False):
                    f.feature = True
            extra = {k: v for k, v in obj.items() if k != "entity"}
            extra["entityName"] = ent.get("name")
            return cls(fields, extra)
        fields = [FeatureField.from_json(d) for d in obj.get("fields", [])]
        return cls(fields, {k: v for k, v in obj.items() if k != "fields"})

    load = from_json

    def to_json(self) -> dict[str, Any]:
        d = {"fields": [f.to_json() for f in self.fields]}
        d.update(self.extra)
        return d

    def dumps(self) -> str:
        return json.dumps(self.to_json(), indent=2)

    # -- chombo FeatureSchema API --------------------------------------------------------------
    def find_class_attr_field(self) -> FeatureField | None:
        for f in self.fields:  # explicit "classAttribute": true (sifarish entity schemas)
            if f.extra.get("classAttribute", False):
                return f
        for f in self.fields:
            if not f.id and not f.feature and f.data_type != "string":
                return f
        for f in self.fields:
            if not f.id and not f.feature:
                return f
        return None

    findClassAttrField = find_class_attr_field

    @property
    def class_field(self) -> FeatureField | None:
        return self.find_class_attr_field()

    @property
    def feature_fields(self) -> list[FeatureField]:
        return [f for f in self.fields if f.feature]

    @property
    def id_field(self) -> FeatureField | None:
        for f in self.fields:
            if f.id:
                return f
        return None

    def find_field_by_ordinal(self, ordinal: int) -> FeatureField:
        for f in self.fields:
            if f.ordinal == ordinal:
                return f
        raise KeyError(f"no field with ordinal {ordinal}")

    def find_field_by_name(self, name: str) -> FeatureField:
        for f in self.fields:
            if f.name == name:
                return f
        raise KeyError(f"no field named {name!r}")

    def __iter__(self):
        return iter(self.fields)

    def __len__(self) -> int:
        return len(self.fields)

"""Params / Transformer / Estimator / Pipeline / PipelineModel (pyspark.ml-compatible).

Persistence follows Spark's ``DefaultParamsWriter``: explicitly set params go to ``paramMap``,
defaults to ``defaultParamMap``; ``PipelineModel`` stores ``stageUids`` and writes each stage to
``stages/{i}_{uid}`` (/root/reference/dialogue_classification_model/metadata/part-00000:1).
Loading dispatches on the JVM class name recorded in each stage's metadata, so a directory saved
by Spark 3.5 (e.g. the shipped ``dialogue_classification_model``) loads unchanged.
"""
from __future__ import annotations

import copy as _copy
import shutil
from pathlib import Path
from typing import Any, Callable, Optional, Sequence

from ..io import spark_format as sf
from .frame import Frame

_REGISTRY: dict[str, type] = {}


def register(java_class: str):
    def deco(cls):
        cls._java_class = java_class
        _REGISTRY[java_class] = cls
        return cls
    return deco


def lookup_class(java_class: str) -> type:
    if java_class not in _REGISTRY:
        raise NotImplementedError(f"no reader for Spark class {java_class}")
    return _REGISTRY[java_class]


class Param:
    def __init__(self, name: str, doc: str = "", default: Any = None, typ: Optional[Callable] = None,
                 has_default: bool = True):
        self.name, self.doc, self.default, self.typ, self.has_default = name, doc, default, typ, has_default

    def convert(self, v):
        if v is None or self.typ is None:
            return v
        if self.typ is float:
            return float(v)
        if self.typ is int:
            return int(v)
        if self.typ is bool:
            return bool(v)
        if self.typ is list:
            return list(v)
        return self.typ(v)


def _cap(name: str) -> str:
    return name[0].upper() + name[1:]


class Params:
    """Param container. Subclasses declare ``_params = [Param(...), ...]`` (inherited and merged).
    ``get<Name>()``/``set<Name>(v)`` accessors are generated like pyspark's."""

    _params: list = []
    _uid_prefix: str = "Params"
    _java_class: str = ""
    _persist_defaults_only: tuple = ()   # params Spark omits from defaultParamMap

    def __init__(self, **kwargs):
        self.uid = kwargs.pop("uid", None) or sf.new_uid(self._uid_prefix)
        self._paramMap: dict = {}
        self._defaultParamMap: dict = {}
        for p in self.params():
            if p.has_default:
                self._defaultParamMap[p.name] = p.default() if callable(p.default) and not isinstance(p.default, type) else p.default
        self._default_hook()
        self.setParams(**kwargs)

    def _default_hook(self) -> None:
        """Per-instance defaults that depend on uid (e.g. ``outputCol = uid + '__output'``)."""

    @classmethod
    def params(cls) -> list:
        seen: dict[str, Param] = {}
        for klass in reversed(cls.__mro__):
            for p in klass.__dict__.get("_params", []):
                seen[p.name] = p
        return list(seen.values())

    @classmethod
    def _param(cls, name: str) -> Param:
        for p in cls.params():
            if p.name == name:
                return p
        raise AttributeError(f"{cls.__name__} has no param {name!r}")

    def setParams(self, **kwargs):  # noqa: N802
        for k, v in kwargs.items():
            if v is not None:
                self.set(k, v)
        return self

    def set(self, name: str, value):
        self._paramMap[name] = self._param(name).convert(value)
        return self

    def clear(self, name: str):
        self._paramMap.pop(name, None)
        return self

    def isSet(self, name: str) -> bool:  # noqa: N802
        return name in self._paramMap

    def isDefined(self, name: str) -> bool:  # noqa: N802
        return name in self._paramMap or name in self._defaultParamMap

    def getOrDefault(self, name: str):  # noqa: N802
        if name in self._paramMap:
            return self._paramMap[name]
        if name in self._defaultParamMap:
            return self._defaultParamMap[name]
        raise KeyError(f"param {name!r} of {self.uid} is not set and has no default")

    def extractParamMap(self) -> dict:  # noqa: N802
        return {**self._defaultParamMap, **self._paramMap}

    def explainParams(self) -> str:  # noqa: N802
        lines = []
        for p in self.params():
            cur = self._paramMap.get(p.name, "undefined")
            lines.append(f"{p.name}: {p.doc} (default: {self._defaultParamMap.get(p.name, 'undefined')}, current: {cur})")
        return "\n".join(lines)

    def copy(self, extra: Optional[dict] = None):
        c = _copy.copy(self)
        c._paramMap = dict(self._paramMap)
        c._defaultParamMap = dict(self._defaultParamMap)
        if extra:
            c.setParams(**extra)
        return c

    def __getattr__(self, item: str):
        if item.startswith("get") and len(item) > 3:
            name = item[3].lower() + item[4:]
            try:
                self._param(name)
            except AttributeError:
                raise AttributeError(item) from None
            return lambda: self.getOrDefault(name)
        if item.startswith("set") and len(item) > 3:
            name = item[3].lower() + item[4:]
            try:
                self._param(name)
            except AttributeError:
                raise AttributeError(item) from None
            return lambda v: self.set(name, v)
        raise AttributeError(item)

    # ------------------------------------------------------------ persistence
    def _json_params(self, m: dict) -> dict:
        out = {}
        for k, v in m.items():
            p = self._param(k) if any(q.name == k for q in self.params()) else None
            if p is not None and p.typ is float and v is not None:
                v = float(v)
            out[k] = v
        return out

    def _metadata_extra(self) -> Optional[dict]:
        return None

    def _save_metadata(self, path) -> None:
        dflt = {k: v for k, v in self._defaultParamMap.items() if k not in self._persist_defaults_only}
        sf.write_metadata(path, self._java_class, self.uid, self._json_params(self._paramMap),
                          self._json_params(dflt), self._metadata_extra())

    def _save_data(self, path) -> None:
        """Stage-specific ``data/`` (models override)."""

    def save(self, path, overwrite: bool = False) -> None:
        p = Path(path)
        if p.exists():
            if not overwrite:
                raise FileExistsError(f"{path} already exists; use write().overwrite().save(path)")
            shutil.rmtree(p)
        self._save_metadata(p)
        self._save_data(p)

    def write(self) -> "_Writer":
        return _Writer(self)

    @classmethod
    def _from_metadata(cls, path, md: dict):
        obj = cls.__new__(cls)
        Params.__init__(obj, uid=md["uid"])
        obj._defaultParamMap.update(md.get("defaultParamMap", {}))
        obj._paramMap.update(md.get("paramMap", {}))
        obj._load_data(path, md)
        return obj

    def _load_data(self, path, md: dict) -> None:
        """Stage-specific data loader (models override)."""

    @classmethod
    def load(cls, path):
        md = sf.read_metadata(path)
        klass = lookup_class(md["class"])
        if cls not in (Params, Transformer, Estimator, Model) and not issubclass(klass, cls):
            raise TypeError(f"{path} holds a {md['class']}, not a {cls.__name__}")
        return klass._from_metadata(path, md)

    @classmethod
    def read(cls):
        return _Reader(cls)


class _Writer:
    def __init__(self, obj):
        self.obj, self._overwrite = obj, False

    def overwrite(self):
        self._overwrite = True
        return self

    def save(self, path):
        self.obj.save(path, overwrite=self._overwrite)


class _Reader:
    def __init__(self, cls):
        self.cls = cls

    def load(self, path):
        return self.cls.load(path)


class Transformer(Params):
    def transform(self, frame: Frame, params: Optional[dict] = None) -> Frame:
        stage = self.copy(params) if params else self
        return stage._transform(frame)

    def _transform(self, frame: Frame) -> Frame:
        raise NotImplementedError


class Estimator(Params):
    def fit(self, frame: Frame, params: Optional[dict] = None):
        stage = self.copy(params) if params else self
        model = stage._fit(frame)
        model.parent = stage
        return model

    def _fit(self, frame: Frame):
        raise NotImplementedError


class Model(Transformer):
    parent = None


class HasInOut:
    _params = [Param("inputCol", "input column name", None, str, has_default=False),
               Param("outputCol", "output column name", None, str)]

    def _default_hook(self) -> None:
        self._defaultParamMap["outputCol"] = f"{self.uid}__output"


# ----------------------------------------------------------------------------- pipelines
@register("org.apache.spark.ml.Pipeline")
class Pipeline(Estimator):
    _uid_prefix = "Pipeline"
    _params = [Param("stages", "pipeline stages", None, list, has_default=False)]

    def __init__(self, stages: Optional[Sequence] = None, **kw):
        super().__init__(**kw)
        if stages is not None:
            self._paramMap["stages"] = list(stages)

    def getStages(self) -> list:  # noqa: N802
        return list(self.getOrDefault("stages"))

    def _fit(self, frame: Frame) -> "PipelineModel":
        stages = self.getStages()
        last_est = max((i for i, s in enumerate(stages) if isinstance(s, Estimator)), default=-1)
        fitted = []
        cur = frame
        for i, s in enumerate(stages):
            if isinstance(s, Estimator):
                m = s.fit(cur)
                fitted.append(m)
                if i < last_est:
                    cur = m.transform(cur)
            else:
                fitted.append(s)
                if i < last_est:
                    cur = s.transform(cur)
        return PipelineModel(fitted, uid=self.uid)

    def _save_metadata(self, path) -> None:
        raise NotImplementedError("saving an unfitted Pipeline is not supported; save the PipelineModel")


@register("org.apache.spark.ml.PipelineModel")
class PipelineModel(Model):
    _uid_prefix = "PipelineModel"

    def __init__(self, stages: Sequence, uid: Optional[str] = None):
        super().__init__(uid=uid)
        self.stages = list(stages)

    def _transform(self, frame: Frame) -> Frame:
        from . import fused

        plan = fused.plan_pipeline(self.stages, frame)
        if plan is not None:
            return plan.run(frame)
        for s in self.stages:
            frame = s.transform(frame)
        return frame

    def compile(self, device=None):
        """Fused serving kernel for text -> prediction (see ``ml.fused.FusedPipeline``)."""
        from . import fused

        return fused.FusedPipeline.from_stages(self.stages, device=device)

    def _save_metadata(self, path) -> None:
        sf.write_metadata(path, self._java_class, self.uid, {"stageUids": [s.uid for s in self.stages]}, {})

    def _save_data(self, path) -> None:
        for i, s in enumerate(self.stages):
            s.save(Path(path) / "stages" / f"{i}_{s.uid}")

    @classmethod
    def _from_metadata(cls, path, md: dict):
        uids = md["paramMap"]["stageUids"]
        stages = []
        for i, uid in enumerate(uids):
            stages.append(Params.load(Path(path) / "stages" / f"{i}_{uid}"))
        return cls(stages, uid=md["uid"])

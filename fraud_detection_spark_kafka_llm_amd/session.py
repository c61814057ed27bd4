"""A ``SparkSession``-shaped entry point without a JVM (R-01, R-21).

Supports the calls the reference makes: ``SparkSession.builder.config(...).appName(...).getOrCreate()``
(/root/reference/fraud_detection_spark.py:23-28, utils/agent_api.py:126, app_ui.py:18),
``createDataFrame`` (pandas or rows + schema), ``read.csv(path, header=True, inferSchema=True)`` and
``stop()``. The session carries the framework config (device, world size) instead of Spark
executors; ``spark.jars.packages`` and other Spark settings are accepted and recorded.
"""
from __future__ import annotations

import threading
from typing import Optional, Sequence

from .ml.frame import Frame
from .utils.config import Config


class _Reader:
    def __init__(self, session: "SparkSession"):
        self.session = session

    def csv(self, path: str, header: bool = True, inferSchema: bool = True, **kw) -> Frame:  # noqa: N803
        import pandas as pd

        df = pd.read_csv(path, header=0 if header else None, dtype=None if inferSchema else str, **kw)
        return Frame.from_pandas(df)


class SparkSession:
    _active: Optional["SparkSession"] = None
    _lock = threading.Lock()

    def __init__(self, app_name: str, conf: dict):
        self.app_name = app_name
        self.conf = dict(conf)
        self.config = Config.from_env()
        self.read = _Reader(self)
        self.stopped = False

    class Builder:
        def __init__(self):
            self._conf: dict = {}
            self._name = "fdx"

        def appName(self, name: str) -> "SparkSession.Builder":  # noqa: N802
            self._name = name
            return self

        def config(self, key=None, value=None, conf=None, **kw) -> "SparkSession.Builder":
            if key is not None:
                self._conf[key] = value
            if conf:
                self._conf.update(conf)
            self._conf.update(kw)
            return self

        def master(self, m: str) -> "SparkSession.Builder":
            self._conf["spark.master"] = m
            return self

        def getOrCreate(self) -> "SparkSession":  # noqa: N802
            with SparkSession._lock:
                s = SparkSession._active
                if s is None or s.stopped:
                    s = SparkSession(self._name, self._conf)
                    SparkSession._active = s
                else:
                    s.conf.update(self._conf)
                return s

    builder = None  # replaced below by a property-like fresh Builder

    def createDataFrame(self, data, schema: Optional[Sequence] = None) -> Frame:  # noqa: N802
        try:
            import pandas as pd

            if isinstance(data, pd.DataFrame):
                if schema is not None:
                    names = [f if isinstance(f, str) else f.name for f in
                             (schema.fields if hasattr(schema, "fields") else schema)]
                    data = data.copy()
                    data.columns = names[: len(data.columns)]
                    for c in names:
                        data[c] = data[c].astype(object).where(data[c].notna(), None).map(
                            lambda v: v if v is None else str(v))
                return Frame.from_pandas(data)
        except ImportError:
            pass
        rows = list(data)
        if schema is None:
            raise ValueError("schema (column names) required for row data")
        names = [f if isinstance(f, str) else f.name for f in (schema.fields if hasattr(schema, "fields") else schema)]
        return Frame.from_records(rows, names)

    @property
    def sparkContext(self):  # noqa: N802
        return self

    def stop(self) -> None:
        self.stopped = True
        with SparkSession._lock:
            if SparkSession._active is self:
                SparkSession._active = None


class _BuilderDescriptor:
    def __get__(self, obj, owner):
        return SparkSession.Builder()


SparkSession.builder = _BuilderDescriptor()

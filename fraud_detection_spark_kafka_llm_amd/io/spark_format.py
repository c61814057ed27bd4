"""Spark ML on-disk persistence without a JVM.

Layout written/read here is byte-compatible with Spark 3.5 ``MLWriter``/``MLReader``:

* ``<dir>/metadata/part-00000``  one compact JSON line (json4s style, Java double formatting)
  with ``class, timestamp, sparkVersion, uid, paramMap, defaultParamMap`` (+ extra keys);
* ``<dir>/data/part-00000-<uuid>-c000.snappy.parquet``  one row group, SNAPPY, whose Arrow
  schema metadata carries ``org.apache.spark.sql.parquet.row.metadata`` (the Spark StructType
  JSON, with ``VectorUDT``/``MatrixUDT`` markers) and ``org.apache.spark.version``;
* an empty ``_SUCCESS`` per directory and a Hadoop checksum sidecar ``.<name>.crc`` per file
  (``b"crc\\0"``, big-endian u32 bytesPerChecksum=512, one big-endian CRC32 per 512-byte chunk).

Reference artefact: /root/reference/dialogue_classification_model/ (metadata JSON at
``metadata/part-00000:1``; IDF/LR parquet schemas verified against it in tests).
"""
from __future__ import annotations

import decimal
import json
import math
import os
import struct
import time
import uuid as _uuid
import zlib
from pathlib import Path
from typing import Any, Iterable

import numpy as np
import pyarrow as pa
import pyarrow.parquet as pq

SPARK_VERSION = "3.5.5"
BYTES_PER_CHECKSUM = 512


# ----------------------------------------------------------------------------- JSON
class JDouble(float):
    """Marks a value that Spark serialises as a JVM double (``1.0``, ``1.0E-6``)."""


def java_double_str(x: float) -> str:
    if math.isnan(x):
        return "NaN"
    if math.isinf(x):
        return "Infinity" if x > 0 else "-Infinity"
    if x == 0.0:
        return "-0.0" if math.copysign(1.0, x) < 0 else "0.0"
    a = abs(x)
    if 1e-3 <= a < 1e7:
        r = repr(float(x))
        if "e" in r or "E" in r:   # defensive; repr is positional in this range
            r = format(float(x), "f")
        return r if "." in r else r + ".0"
    d = decimal.Decimal(repr(float(a))).normalize()
    sign, digits, exp = d.as_tuple()
    ds = "".join(map(str, digits))
    e10 = exp + len(ds) - 1
    mant = ds[0] + "." + (ds[1:] if len(ds) > 1 else "0")
    return ("-" if x < 0 else "") + f"{mant}E{e10}"


def _enc(v: Any) -> str:
    if isinstance(v, bool):
        return "true" if v else "false"
    if v is None:
        return "null"
    if isinstance(v, (float, np.floating)):
        return java_double_str(float(v))
    if isinstance(v, (int, np.integer)):
        return str(int(v))
    if isinstance(v, str):
        return json.dumps(v, ensure_ascii=False)
    if isinstance(v, dict):
        return "{" + ",".join(f"{json.dumps(str(k), ensure_ascii=False)}:{_enc(x)}" for k, x in v.items()) + "}"
    if isinstance(v, (list, tuple)):
        return "[" + ",".join(_enc(x) for x in v) + "]"
    raise TypeError(f"cannot serialise {type(v)}")


def spark_json_dumps(obj: Any) -> str:
    """Compact JSON with Java double rendering (json4s ``compact(render(...))``)."""
    return _enc(obj)


# ----------------------------------------------------------------------------- CRC / files
def crc_bytes(data: bytes) -> bytes:
    out = [b"crc\x00", struct.pack(">I", BYTES_PER_CHECKSUM)]
    for i in range(0, len(data), BYTES_PER_CHECKSUM):
        out.append(struct.pack(">I", zlib.crc32(data[i:i + BYTES_PER_CHECKSUM]) & 0xFFFFFFFF))
    return b"".join(out)


def write_file_with_crc(path: Path, data: bytes) -> None:
    path = Path(path)
    path.parent.mkdir(parents=True, exist_ok=True)
    path.write_bytes(data)
    (path.parent / f".{path.name}.crc").write_bytes(crc_bytes(data))


def mark_success(directory: Path) -> None:
    write_file_with_crc(Path(directory) / "_SUCCESS", b"")


def verify_crc(path: Path) -> bool:
    path = Path(path)
    crc = path.parent / f".{path.name}.crc"
    if not crc.exists():
        return False
    return crc.read_bytes() == crc_bytes(path.read_bytes())


def verify_tree(root: Path) -> list[str]:
    """Return the list of files under ``root`` whose CRC sidecar is missing or wrong."""
    bad = []
    for dirpath, _, files in os.walk(root):
        for f in files:
            if f.endswith(".crc"):
                continue
            p = Path(dirpath) / f
            if not verify_crc(p):
                bad.append(str(p))
    return bad


# ----------------------------------------------------------------------------- metadata
def new_uid(prefix: str) -> str:
    return f"{prefix}_{_uuid.uuid4().hex[:12]}"


def write_metadata(path: str | os.PathLike, cls: str, uid: str, param_map: dict, default_param_map: dict,
                   extra: dict | None = None, timestamp: int | None = None) -> None:
    md = {
        "class": cls,
        "timestamp": int(timestamp if timestamp is not None else time.time() * 1000),
        "sparkVersion": SPARK_VERSION,
        "uid": uid,
        "paramMap": param_map,
        "defaultParamMap": default_param_map,
    }
    if extra:
        md.update(extra)
    d = Path(path) / "metadata"
    write_file_with_crc(d / "part-00000", (spark_json_dumps(md) + "\n").encode("utf-8"))
    mark_success(d)


def read_metadata(path: str | os.PathLike) -> dict:
    d = Path(path) / "metadata"
    parts = sorted(p for p in d.iterdir() if p.name.startswith("part-"))
    if not parts:
        raise FileNotFoundError(f"no metadata part file under {d}")
    return json.loads(parts[0].read_text(encoding="utf-8").splitlines()[0])


# ----------------------------------------------------------------------------- schemas
def _sf(name: str, typ: Any, nullable: bool) -> dict:
    return {"name": name, "type": typ, "nullable": nullable, "metadata": {}}


def _arr(elem: str) -> dict:
    return {"type": "array", "elementType": elem, "containsNull": False}


VECTOR_SQL = {"type": "struct", "fields": [
    _sf("type", "byte", False), _sf("size", "integer", True),
    _sf("indices", _arr("integer"), True), _sf("values", _arr("double"), True)]}
MATRIX_SQL = {"type": "struct", "fields": [
    _sf("type", "byte", False), _sf("numRows", "integer", False), _sf("numCols", "integer", False),
    _sf("colPtrs", _arr("integer"), True), _sf("rowIndices", _arr("integer"), True),
    _sf("values", _arr("double"), True), _sf("isTransposed", "boolean", False)]}
VECTOR_UDT = {"type": "udt", "class": "org.apache.spark.ml.linalg.VectorUDT",
              "pyClass": "pyspark.ml.linalg.VectorUDT", "sqlType": VECTOR_SQL}
MATRIX_UDT = {"type": "udt", "class": "org.apache.spark.ml.linalg.MatrixUDT",
              "pyClass": "pyspark.ml.linalg.MatrixUDT", "sqlType": MATRIX_SQL}

_LIST_I32 = pa.list_(pa.field("element", pa.int32(), nullable=False))
_LIST_I64 = pa.list_(pa.field("element", pa.int64(), nullable=False))
_LIST_F64 = pa.list_(pa.field("element", pa.float64(), nullable=False))
_LIST_STR = pa.list_(pa.field("element", pa.string(), nullable=True))
VECTOR_ARROW = pa.struct([pa.field("type", pa.int8(), False), pa.field("size", pa.int32(), True),
                          pa.field("indices", _LIST_I32, True), pa.field("values", _LIST_F64, True)])
MATRIX_ARROW = pa.struct([pa.field("type", pa.int8(), False), pa.field("numRows", pa.int32(), False),
                          pa.field("numCols", pa.int32(), False), pa.field("colPtrs", _LIST_I32, True),
                          pa.field("rowIndices", _LIST_I32, True), pa.field("values", _LIST_F64, True),
                          pa.field("isTransposed", pa.bool_(), False)])

# Spark simple type name -> arrow type
_SIMPLE = {"integer": pa.int32(), "long": pa.int64(), "double": pa.float64(), "boolean": pa.bool_(),
           "string": pa.string(), "byte": pa.int8()}


class Field:
    """One column of a Spark-written parquet file: Spark type JSON + matching Arrow field."""

    def __init__(self, name: str, spark_type: Any, arrow_type: pa.DataType, nullable: bool):
        self.name, self.spark_type, self.arrow_type, self.nullable = name, spark_type, arrow_type, nullable

    @classmethod
    def simple(cls, name: str, t: str, nullable: bool = False) -> "Field":
        return cls(name, t, _SIMPLE[t], nullable)

    @classmethod
    def array(cls, name: str, elem: str, nullable: bool = True, contains_null: bool = False) -> "Field":
        at = pa.list_(pa.field("element", _SIMPLE[elem], nullable=contains_null))
        return cls(name, {"type": "array", "elementType": elem, "containsNull": contains_null}, at, nullable)

    @classmethod
    def vector(cls, name: str, nullable: bool = True) -> "Field":
        return cls(name, VECTOR_UDT, VECTOR_ARROW, nullable)

    @classmethod
    def matrix(cls, name: str, nullable: bool = True) -> "Field":
        return cls(name, MATRIX_UDT, MATRIX_ARROW, nullable)

    @classmethod
    def struct(cls, name: str, fields: list["Field"], nullable: bool = True) -> "Field":
        st = {"type": "struct", "fields": [_sf(f.name, f.spark_type, f.nullable) for f in fields]}
        at = pa.struct([pa.field(f.name, f.arrow_type, f.nullable) for f in fields])
        return cls(name, st, at, nullable)


def write_data_parquet(path: str | os.PathLike, fields: list[Field], rows: list[dict], subdir: str = "data") -> Path:
    """Write ``rows`` as a Spark-style single-file parquet directory ``<path>/<subdir>``."""
    schema_json = {"type": "struct", "fields": [_sf(f.name, f.spark_type, f.nullable) for f in fields]}
    schema = pa.schema([pa.field(f.name, f.arrow_type, f.nullable) for f in fields],
                       metadata={"org.apache.spark.version": SPARK_VERSION,
                                 "org.apache.spark.sql.parquet.row.metadata": json.dumps(schema_json, separators=(",", ":"))})
    cols = {f.name: [r[f.name] for r in rows] for f in fields}
    table = pa.table({f.name: pa.array(cols[f.name], type=f.arrow_type) for f in fields}, schema=schema)
    d = Path(path) / subdir
    d.mkdir(parents=True, exist_ok=True)
    name = f"part-00000-{_uuid.uuid4()}-c000.snappy.parquet"
    sink = pa.BufferOutputStream()
    pq.write_table(table, sink, compression="snappy", row_group_size=max(1, len(rows)),
                   use_dictionary=False, write_statistics=True)
    write_file_with_crc(d / name, sink.getvalue().to_pybytes())
    mark_success(d)
    return d / name


def read_data_parquet(path: str | os.PathLike, subdir: str = "data") -> pa.Table:
    d = Path(path) / subdir
    parts = sorted(p for p in d.iterdir() if p.name.startswith("part-") and p.name.endswith(".parquet"))
    if not parts:
        raise FileNotFoundError(f"no parquet part under {d}")
    tables = [pq.read_table(p) for p in parts]
    return pa.concat_tables(tables) if len(tables) > 1 else tables[0]


def spark_schema_of(path: str | os.PathLike, subdir: str = "data") -> dict:
    d = Path(path) / subdir
    part = next(p for p in sorted(d.iterdir()) if p.name.endswith(".parquet"))
    md = pq.ParquetFile(part).schema_arrow.metadata or {}
    return json.loads(md[b"org.apache.spark.sql.parquet.row.metadata"])


# ----------------------------------------------------------------------------- UDT values
def dense_vector(values: Iterable[float]) -> dict:
    return {"type": 1, "size": None, "indices": None, "values": [float(v) for v in values]}


def sparse_vector(size: int, indices: Iterable[int], values: Iterable[float]) -> dict:
    return {"type": 0, "size": int(size), "indices": [int(i) for i in indices], "values": [float(v) for v in values]}


def decode_vector(v: dict, size_hint: int | None = None) -> np.ndarray:
    if v["type"] == 1:
        return np.asarray(v["values"], dtype=np.float64)
    out = np.zeros(int(v["size"]), dtype=np.float64)
    out[np.asarray(v["indices"], dtype=np.int64)] = np.asarray(v["values"], dtype=np.float64)
    return out


def dense_matrix(arr: np.ndarray) -> dict:
    arr = np.asarray(arr, dtype=np.float64)
    return {"type": 1, "numRows": int(arr.shape[0]), "numCols": int(arr.shape[1]), "colPtrs": None,
            "rowIndices": None, "values": arr.flatten(order="F").tolist(), "isTransposed": False}


def sparse_matrix_row_major(arr: np.ndarray) -> dict:
    """Spark ``Matrix.compressed`` of a row-major (isTransposed=true) CSR, as LR persists it."""
    arr = np.asarray(arr, dtype=np.float64)
    rows, cols = arr.shape
    ptr, idx, val = [0], [], []
    for r in range(rows):
        nz = np.nonzero(arr[r])[0]
        idx.extend(int(i) for i in nz)
        val.extend(float(v) for v in arr[r, nz])
        ptr.append(len(idx))
    return {"type": 0, "numRows": rows, "numCols": cols, "colPtrs": ptr, "rowIndices": idx, "values": val,
            "isTransposed": True}


def decode_matrix(m: dict) -> np.ndarray:
    rows, cols = int(m["numRows"]), int(m["numCols"])
    tr = bool(m["isTransposed"])
    if m["type"] == 1:
        vals = np.asarray(m["values"], dtype=np.float64)
        return vals.reshape((rows, cols)) if tr else vals.reshape((cols, rows)).T.copy()
    out = np.zeros((rows, cols), dtype=np.float64)
    ptr = m["colPtrs"]
    idx, vals = m["rowIndices"], m["values"]
    major = rows if tr else cols
    for a in range(major):
        for k in range(ptr[a], ptr[a + 1]):
            if tr:
                out[a, idx[k]] = vals[k]
            else:
                out[idx[k], a] = vals[k]
    return out

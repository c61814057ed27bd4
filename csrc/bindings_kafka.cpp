// Kafka client-API glue of the streaming engine (stream/engine.py), in C++ over the CPython API.
//
// A confluent_kafka consumer hands out one Message object per record and a producer takes one
// produce() call per record: with a real librdkafka client there is no columnar path, so the
// per-record work has to leave Python bytecode. pack_messages walks a consumed list once (error,
// topic, partition, key, value, offset, timestamp of every message) into columnar buffers;
// produce_each issues the per-record produce calls of one output segment from a C loop, serving
// delivery reports when the local queue is full (BufferError), like the Python loop it replaces.
#include <torch/extension.h>
#include <pybind11/numpy.h>

#include <cstring>
#include <string>
#include <utility>
#include <vector>

namespace {

namespace py = pybind11;

struct Names {
  PyObject *error, *topic, *partition, *key, *value, *offset, *timestamp, *produce, *poll, *on_delivery;
  Names() {
    error = PyUnicode_InternFromString("error");
    topic = PyUnicode_InternFromString("topic");
    partition = PyUnicode_InternFromString("partition");
    key = PyUnicode_InternFromString("key");
    value = PyUnicode_InternFromString("value");
    offset = PyUnicode_InternFromString("offset");
    timestamp = PyUnicode_InternFromString("timestamp");
    produce = PyUnicode_InternFromString("produce");
    poll = PyUnicode_InternFromString("poll");
    on_delivery = PyUnicode_InternFromString("on_delivery");
  }
};

const Names& names() {
  static Names* n = new Names();   // interned for the process lifetime
  return *n;
}

PyObject* call0(PyObject* o, PyObject* name) { return PyObject_CallMethodObjArgs(o, name, nullptr); }

// bytes / bytearray / str / None -> appended to buf; returns false for None
bool append_bytes(PyObject* v, std::vector<uint8_t>& buf) {
  if (v == Py_None) return false;
  char* p = nullptr;
  Py_ssize_t n = 0;
  if (PyBytes_Check(v)) {
    PyBytes_AsStringAndSize(v, &p, &n);
  } else if (PyUnicode_Check(v)) {
    p = const_cast<char*>(PyUnicode_AsUTF8AndSize(v, &n));
    if (!p) throw py::error_already_set();
  } else if (PyByteArray_Check(v)) {
    p = PyByteArray_AsString(v);
    n = PyByteArray_Size(v);
  } else {
    throw py::type_error("message key/value must be bytes, str or None");
  }
  buf.insert(buf.end(), reinterpret_cast<uint8_t*>(p), reinterpret_cast<uint8_t*>(p) + n);
  return true;
}

template <class T>
py::array_t<T> to_array(const std::vector<T>& v) {
  py::array_t<T> a((py::ssize_t)v.size());
  if (!v.empty()) std::memcpy(a.mutable_data(), v.data(), v.size() * sizeof(T));
  return a;
}

// -> (part_of int32[n], parts [(topic, partition)], keys u8, key_off i64[n+1], null_keys u8[n],
//     values u8, val_off i64[n+1], offsets i64[n], ts_ms i64[n], errors [(index, error)])
// over the messages without an error; n counts those.
py::tuple pack_messages(py::list msgs) {
  const Names& N = names();
  const Py_ssize_t m = PyList_GET_SIZE(msgs.ptr());
  std::vector<int32_t> part_of;
  std::vector<std::pair<std::string, int64_t>> parts;
  py::list parts_out, errors;
  std::vector<uint8_t> keys, vals, nulls;
  std::vector<int64_t> koff{0}, voff{0}, offs, ts;
  part_of.reserve(m);
  offs.reserve(m);
  ts.reserve(m);
  koff.reserve(m + 1);
  voff.reserve(m + 1);
  nulls.reserve(m);
  std::string last_topic;
  int64_t last_part = -1;
  int32_t last_idx = -1;
  for (Py_ssize_t i = 0; i < m; ++i) {
    PyObject* msg = PyList_GET_ITEM(msgs.ptr(), i);
    py::object err = py::reinterpret_steal<py::object>(call0(msg, N.error));
    if (!err) throw py::error_already_set();
    if (!err.is_none()) {
      errors.append(py::make_tuple(i, err));
      continue;
    }
    py::object t = py::reinterpret_steal<py::object>(call0(msg, N.topic));
    py::object p = py::reinterpret_steal<py::object>(call0(msg, N.partition));
    if (!t || !p) throw py::error_already_set();
    const std::string topic = t.cast<std::string>();
    const int64_t part = p.cast<int64_t>();
    if (last_idx < 0 || part != last_part || topic != last_topic) {
      last_idx = -1;
      for (size_t k = 0; k < parts.size(); ++k)
        if (parts[k].second == part && parts[k].first == topic) last_idx = (int32_t)k;
      if (last_idx < 0) {
        last_idx = (int32_t)parts.size();
        parts.emplace_back(topic, part);
        parts_out.append(py::make_tuple(t, part));
      }
      last_topic = topic;
      last_part = part;
    }
    part_of.push_back(last_idx);
    py::object k = py::reinterpret_steal<py::object>(call0(msg, N.key));
    py::object v = py::reinterpret_steal<py::object>(call0(msg, N.value));
    py::object o = py::reinterpret_steal<py::object>(call0(msg, N.offset));
    py::object ts_obj = py::reinterpret_steal<py::object>(call0(msg, N.timestamp));
    if (!k || !v || !o || !ts_obj) throw py::error_already_set();
    nulls.push_back(append_bytes(k.ptr(), keys) ? 0 : 1);
    koff.push_back((int64_t)keys.size());
    append_bytes(v.ptr(), vals);
    voff.push_back((int64_t)vals.size());
    offs.push_back(o.cast<int64_t>());
    int64_t tms = -1;
    if (PyTuple_Check(ts_obj.ptr()) && PyTuple_GET_SIZE(ts_obj.ptr()) == 2) {
      const long kind = PyLong_AsLong(PyTuple_GET_ITEM(ts_obj.ptr(), 0));
      if (kind != 0) tms = PyLong_AsLongLong(PyTuple_GET_ITEM(ts_obj.ptr(), 1));
      if (PyErr_Occurred()) throw py::error_already_set();
    }
    ts.push_back(tms);
  }
  return py::make_tuple(to_array(part_of), parts_out, to_array(keys), to_array(koff), to_array(nulls), to_array(vals),
                        to_array(voff), to_array(offs), to_array(ts), errors);
}

// producer.produce(topic, value=v_i, key=k_i, on_delivery=cb) for the n records of one segment
// (keys[koff[i]:koff[i+1]], None where null_keys[i]); a BufferError (local queue full) serves
// delivery reports with producer.poll(0.05) and retries; any other error is reported to cb(err,
// None) for that record. Returns the number of records handed to the producer.
int64_t produce_each(py::object producer, py::object topic, py::array_t<uint8_t> keys, py::array_t<int64_t> koff,
                     py::object null_keys, py::array_t<uint8_t> vals, py::array_t<int64_t> voff, py::object cb) {
  const Names& N = names();
  py::object produce = producer.attr(N.produce);
  py::object poll = producer.attr(N.poll);
  const int64_t n = voff.size() - 1;
  const uint8_t* kb = keys.data();
  const int64_t* ko = koff.data();
  const uint8_t* vb = vals.data();
  const int64_t* vo = voff.data();
  const uint8_t* nk = nullptr;
  py::array_t<uint8_t> nk_arr;
  if (!null_keys.is_none()) {
    nk_arr = py::array_t<uint8_t>::ensure(null_keys);
    nk = nk_arr.data();
  }
  py::tuple args = py::make_tuple(topic);
  py::dict kw;
  kw[N.on_delivery] = cb;
  int64_t sent = 0;
  for (int64_t i = 0; i < n; ++i) {
    py::object kobj = (nk && nk[i]) ? py::none()
                                    : py::reinterpret_steal<py::object>(PyBytes_FromStringAndSize(
                                          reinterpret_cast<const char*>(kb + ko[i]), ko[i + 1] - ko[i]));
    py::object vobj = py::reinterpret_steal<py::object>(
        PyBytes_FromStringAndSize(reinterpret_cast<const char*>(vb + vo[i]), vo[i + 1] - vo[i]));
    kw[N.key] = kobj;
    kw[N.value] = vobj;
    while (true) {
      PyObject* r = PyObject_Call(produce.ptr(), args.ptr(), kw.ptr());
      if (r) {
        Py_DECREF(r);
        ++sent;
        break;
      }
      if (PyErr_ExceptionMatches(PyExc_BufferError)) {
        PyErr_Clear();
        py::object pr = poll(0.05);
        continue;
      }
      PyObject *type, *value, *tb;
      PyErr_Fetch(&type, &value, &tb);
      PyErr_NormalizeException(&type, &value, &tb);
      py::object e = py::reinterpret_steal<py::object>(value ? value : (Py_INCREF(Py_None), Py_None));
      Py_XDECREF(type);
      Py_XDECREF(tb);
      cb(e, py::none());
      break;
    }
  }
  return sent;
}

}  // namespace

void register_kafka_ops(pybind11::module& m) {
  m.def("pack_messages", &pack_messages, "consumed Message list -> columnar buffers (one pass, C loop)");
  m.def("produce_each", &produce_each, "per-record produce of one output segment from a C loop");
}

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

PyObject* call0(PyObject* o, PyObject* name) {
  return PyObject_VectorcallMethod(name, &o, 1 | PY_VECTORCALL_ARGUMENTS_OFFSET, nullptr);
}

// the in-memory broker's Message class (a 7-tuple: topic, partition, offset, key, value, error,
// timestamp ms), registered by install_message_accessors: pack_messages reads its items directly
PyTypeObject* g_message_type = nullptr;

template <class T>
py::array_t<T> to_array(const std::vector<T>& v) {
  py::array_t<T> a((py::ssize_t)v.size());
  if (!v.empty()) std::memcpy(a.mutable_data(), v.data(), v.size() * sizeof(T));
  return a;
}

// bytes / bytearray / str -> (pointer, size); None -> (nullptr, -1)
std::pair<const char*, Py_ssize_t> byte_view(PyObject* v) {
  if (v == Py_None) return {nullptr, -1};
  if (PyBytes_Check(v)) return {PyBytes_AS_STRING(v), PyBytes_GET_SIZE(v)};
  if (PyByteArray_Check(v)) return {PyByteArray_AS_STRING(v), PyByteArray_GET_SIZE(v)};
  if (PyUnicode_Check(v)) {
    Py_ssize_t n = 0;
    const char* p = PyUnicode_AsUTF8AndSize(v, &n);
    if (!p) throw py::error_already_set();
    return {p, n};
  }
  throw py::type_error("message key/value must be bytes, str or None");
}

// -> (part_of int32[n], parts [(topic, partition)], keys u8, key_off i64[n+1], null_keys u8[n],
//     values u8, val_off i64[n+1], offsets i64[n], ts_ms i64[n], errors [(index, error)])
// over the messages without an error; n counts those. by_ref: values is a list of the messages'
// value objects (val_off still counts their bytes), for a consumer that reads them in place
// (extract_json_field_refs) instead of packing them. Two passes: the first reads every
// message's fields (the in-memory broker's Message items directly, other classes through their
// methods) and sizes the buffers, the second copies the bytes once into the final arrays (a
// growing vector plus a copy into numpy faulted in ~64 MB of fresh pages per 16K 2-KB records).
py::tuple pack_messages(py::list msgs, py::object vals_buf, bool by_ref) {
  const Names& N = names();
  const Py_ssize_t m = PyList_GET_SIZE(msgs.ptr());
  struct Rec {
    PyObject* k;
    PyObject* v;
    int64_t off, ts;
  };
  std::vector<Rec> recs;
  std::vector<py::object> hold;          // references owned here (fields read through methods)
  std::vector<int32_t> part_of;
  std::vector<std::pair<std::string, int64_t>> parts;
  py::list parts_out, errors;
  recs.reserve(m);
  part_of.reserve(m);
  std::string last_topic;
  py::object last_topic_obj;
  int64_t last_part = -1;
  int32_t last_idx = -1;
  size_t kbytes = 0, vbytes = 0;
  for (Py_ssize_t i = 0; i < m; ++i) {
    PyObject* msg = PyList_GET_ITEM(msgs.ptr(), i);
    const bool direct = g_message_type && Py_TYPE(msg) == g_message_type && PyTuple_GET_SIZE(msg) == 7;
    py::object err = direct ? py::reinterpret_borrow<py::object>(PyTuple_GET_ITEM(msg, 5))
                            : py::reinterpret_steal<py::object>(call0(msg, N.error));
    if (!err) throw py::error_already_set();
    if (!err.is_none()) {
      errors.append(py::make_tuple(i, err));
      continue;
    }
    py::object t = direct ? py::reinterpret_borrow<py::object>(PyTuple_GET_ITEM(msg, 0))
                          : py::reinterpret_steal<py::object>(call0(msg, N.topic));
    py::object p = direct ? py::reinterpret_borrow<py::object>(PyTuple_GET_ITEM(msg, 1))
                          : py::reinterpret_steal<py::object>(call0(msg, N.partition));
    if (!t || !p) throw py::error_already_set();
    const int64_t part = p.cast<int64_t>();
    // consecutive messages share the topic object: compare it before converting the string
    const bool same_topic = t.ptr() == last_topic_obj.ptr();
    const std::string topic = same_topic ? last_topic : t.cast<std::string>();
    last_topic_obj = t;
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
    Rec r{};
    if (direct) {                 // borrowed items of the in-memory Message (the list keeps them)
      PyObject* ts_item = PyTuple_GET_ITEM(msg, 6);
      r.k = PyTuple_GET_ITEM(msg, 3);
      r.v = PyTuple_GET_ITEM(msg, 4);
      r.off = (int64_t)PyLong_AsLongLong(PyTuple_GET_ITEM(msg, 2));
      r.ts = ts_item == Py_None ? -1 : (int64_t)PyLong_AsLongLong(ts_item);
      if (PyErr_Occurred()) throw py::error_already_set();
    } else {
      py::object k = py::reinterpret_steal<py::object>(call0(msg, N.key));
      py::object v = py::reinterpret_steal<py::object>(call0(msg, N.value));
      py::object o = py::reinterpret_steal<py::object>(call0(msg, N.offset));
      py::object ts_obj = py::reinterpret_steal<py::object>(call0(msg, N.timestamp));
      if (!k || !v || !o || !ts_obj) throw py::error_already_set();
      r.k = k.ptr();
      r.v = v.ptr();
      r.off = o.cast<int64_t>();
      r.ts = -1;
      if (PyTuple_Check(ts_obj.ptr()) && PyTuple_GET_SIZE(ts_obj.ptr()) == 2) {
        const long kind = PyLong_AsLong(PyTuple_GET_ITEM(ts_obj.ptr(), 0));
        if (kind != 0) r.ts = PyLong_AsLongLong(PyTuple_GET_ITEM(ts_obj.ptr(), 1));
        if (PyErr_Occurred()) throw py::error_already_set();
      }
      hold.push_back(std::move(k));
      hold.push_back(std::move(v));
    }
    const auto kv = byte_view(r.k), vv = byte_view(r.v);
    kbytes += kv.second > 0 ? (size_t)kv.second : 0;
    vbytes += vv.second > 0 ? (size_t)vv.second : 0;
    recs.push_back(r);
  }
  const py::ssize_t n = (py::ssize_t)recs.size();
  py::array_t<uint8_t> keys((py::ssize_t)kbytes), nulls(n);
  py::list refs;
  if (by_ref) {                  // values stay in their own bytes objects: a list of references
    refs = py::list(n);
    for (py::ssize_t i = 0; i < n; ++i) {
      PyObject* v = recs[i].v;
      if (v != Py_None && !PyBytes_Check(v)) throw py::type_error("by_ref: message values must be bytes or None");
      Py_INCREF(v);
      PyList_SET_ITEM(refs.ptr(), i, v);
    }
    vbytes = 0;
  }
  // values: into the caller's reusable buffer when it is large enough (a view of it is returned;
  // fresh 32-MB arrays are page-faulted in on every batch), else a new array
  bool reuse = false;
  py::array_t<uint8_t, py::array::c_style> given;
  if (!vals_buf.is_none()) {
    given = py::array_t<uint8_t, py::array::c_style>::ensure(vals_buf);
    if (!given) throw py::type_error("vals_buf must be a contiguous uint8 array");
    reuse = (size_t)given.size() >= vbytes && given.writeable();
  }
  py::array_t<uint8_t> vals = reuse ? py::array_t<uint8_t>(given) : py::array_t<uint8_t>((py::ssize_t)vbytes);
  py::array_t<int64_t> koff(n + 1), voff(n + 1), offs(n), ts(n);
  uint8_t *kp = keys.mutable_data(), *vp = vals.mutable_data(), *np_ = nulls.mutable_data();
  int64_t *ko = koff.mutable_data(), *vo = voff.mutable_data(), *op = offs.mutable_data(), *tp = ts.mutable_data();
  size_t kpos = 0, vpos = 0;
  ko[0] = vo[0] = 0;
  for (py::ssize_t i = 0; i < n; ++i) {
    const auto kv = byte_view(recs[i].k), vv = byte_view(recs[i].v);
    np_[i] = kv.first ? 0 : 1;
    if (kv.second > 0) std::memcpy(kp + kpos, kv.first, (size_t)kv.second), kpos += (size_t)kv.second;
    if (vv.second > 0) {
      if (!by_ref) std::memcpy(vp + vpos, vv.first, (size_t)vv.second);
      vpos += (size_t)vv.second;
    }
    ko[i + 1] = (int64_t)kpos;
    vo[i + 1] = (int64_t)vpos;
    op[i] = recs[i].off;
    tp[i] = recs[i].ts;
  }
  py::object vals_out = by_ref ? py::object(refs)
                       : (size_t)vals.size() == vbytes ? py::object(vals)
                                                       : vals[py::slice(0, (py::ssize_t)vbytes, 1)];
  return py::make_tuple(to_array(part_of), parts_out, keys, koff, nulls, vals_out, voff, offs, ts, errors);
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
  // vectorcall: produce(topic, value=, key=, on_delivery=) without a kwargs dict per record
  py::tuple kwnames = py::make_tuple(py::reinterpret_borrow<py::object>(N.value),
                                     py::reinterpret_borrow<py::object>(N.key),
                                     py::reinterpret_borrow<py::object>(N.on_delivery));
  int64_t sent = 0;
  for (int64_t i = 0; i < n; ++i) {
    if (i && (i & 255) == 0) {                    // let the reader / client threads run between records
      PyThreadState* ts = PyEval_SaveThread();
      PyEval_RestoreThread(ts);
    }
    py::object kobj = (nk && nk[i]) ? py::none()
                                    : py::reinterpret_steal<py::object>(PyBytes_FromStringAndSize(
                                          reinterpret_cast<const char*>(kb + ko[i]), ko[i + 1] - ko[i]));
    py::object vobj = py::reinterpret_steal<py::object>(
        PyBytes_FromStringAndSize(reinterpret_cast<const char*>(vb + vo[i]), vo[i + 1] - vo[i]));
    PyObject* vargs[4] = {topic.ptr(), vobj.ptr(), kobj.ptr(), cb.ptr()};
    while (true) {
      PyObject* r = PyObject_Vectorcall(produce.ptr(), vargs, 1, kwnames.ptr());
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

// ------------------------------------------------------------------------------------------------
// DeliveryCounter(n, done): the per-record on_delivery callback of one output segment. Each call
// (err, msg) counts one report; the first error is kept; the n-th call runs done(err or None).
// A C callable: librdkafka-speed reports do not pay a Python frame per record.
struct DeliveryCounter {
  PyObject_HEAD
  int64_t left;
  PyObject* done;
  PyObject* err;
};

void dc_dealloc(PyObject* self) {
  auto* d = reinterpret_cast<DeliveryCounter*>(self);
  Py_XDECREF(d->done);
  Py_XDECREF(d->err);
  Py_TYPE(self)->tp_free(self);
}

int dc_init(PyObject* self, PyObject* args, PyObject* kw) {
  auto* d = reinterpret_cast<DeliveryCounter*>(self);
  long long n = 0;
  PyObject* done = nullptr;
  if (!PyArg_ParseTuple(args, "LO", &n, &done)) return -1;
  Py_INCREF(done);
  Py_XSETREF(d->done, done);
  Py_CLEAR(d->err);
  d->left = n;
  return 0;
}

PyObject* dc_call(PyObject* self, PyObject* args, PyObject* kw) {
  auto* d = reinterpret_cast<DeliveryCounter*>(self);
  PyObject* err = Py_None;
  PyObject* msg = Py_None;
  if (!PyArg_UnpackTuple(args, "DeliveryCounter", 0, 2, &err, &msg)) return nullptr;
  if (err != Py_None && d->err == nullptr) {
    Py_INCREF(err);
    d->err = err;
  }
  if (--d->left == 0) {
    PyObject* r = PyObject_CallOneArg(d->done, d->err ? d->err : Py_None);
    if (!r) return nullptr;
    Py_DECREF(r);
  }
  Py_RETURN_NONE;
}

PyObject* dc_left(PyObject* self, void*) { return PyLong_FromLongLong(reinterpret_cast<DeliveryCounter*>(self)->left); }

PyGetSetDef dc_getset[] = {{"left", dc_left, nullptr, nullptr, nullptr}, {nullptr, nullptr, nullptr, nullptr, nullptr}};

PyTypeObject DeliveryCounterType = [] {
  PyTypeObject t{PyVarObject_HEAD_INIT(nullptr, 0)};
  t.tp_name = "fdx.DeliveryCounter";
  t.tp_basicsize = sizeof(DeliveryCounter);
  t.tp_flags = Py_TPFLAGS_DEFAULT;
  t.tp_new = PyType_GenericNew;
  t.tp_init = dc_init;
  t.tp_dealloc = dc_dealloc;
  t.tp_call = dc_call;
  t.tp_getset = dc_getset;
  t.tp_doc = "per-record delivery callback counting one segment's reports";
  return t;
}();

// ------------------------------------------------------------------------------------------------
// C-level accessors for the in-memory broker's Message (a tuple subclass): method descriptors,
// so msg.value() etc. cost a C call like cimpl.Message's instead of a Python frame.
template <int I>
PyObject* tuple_get(PyObject* self, PyObject*) {
  PyObject* o = PyTuple_GET_ITEM(self, I);
  Py_INCREF(o);
  return o;
}
PyObject* tuple_ts(PyObject* self, PyObject*) { return Py_BuildValue("(iO)", 1, PyTuple_GET_ITEM(self, 6)); }

PyMethodDef message_defs[] = {
    {"topic", tuple_get<0>, METH_NOARGS, "topic"},     {"partition", tuple_get<1>, METH_NOARGS, "partition"},
    {"offset", tuple_get<2>, METH_NOARGS, "offset"},   {"key", tuple_get<3>, METH_NOARGS, "key"},
    {"value", tuple_get<4>, METH_NOARGS, "value"},     {"error", tuple_get<5>, METH_NOARGS, "error"},
    {"timestamp", tuple_ts, METH_NOARGS, "timestamp"}, {nullptr, nullptr, 0, nullptr}};

void install_message_accessors(py::object cls) {
  if (!PyType_Check(cls.ptr()) || !PyType_IsSubtype(reinterpret_cast<PyTypeObject*>(cls.ptr()), &PyTuple_Type))
    throw py::type_error("expected a tuple subclass");
  for (PyMethodDef* d = message_defs; d->ml_name; ++d) {
    PyObject* descr = PyDescr_NewMethod(reinterpret_cast<PyTypeObject*>(cls.ptr()), d);
    if (!descr || PyObject_SetAttrString(cls.ptr(), d->ml_name, descr) < 0) {
      Py_XDECREF(descr);
      throw py::error_already_set();
    }
    Py_DECREF(descr);
  }
  g_message_type = reinterpret_cast<PyTypeObject*>(cls.ptr());
  Py_INCREF(cls.ptr());          // kept for the process lifetime
}

PyObject* new_message(PyObject* cls, PyObject* topic, PyObject* part, PyObject* off, PyObject* key, PyObject* value,
                      PyObject* ts) {
  PyObject* m = reinterpret_cast<PyTypeObject*>(cls)->tp_alloc(reinterpret_cast<PyTypeObject*>(cls), 7);
  if (!m) return nullptr;
  PyObject* items[7] = {topic, part, off, key, value, Py_None, ts};
  for (int i = 0; i < 7; ++i) {
    if (i != 2 && i != 6) Py_INCREF(items[i]);
    PyTuple_SET_ITEM(m, i, items[i]);
  }
  // only str / int / bytes / None inside: no reference cycle can pass through a Message, so the
  // collector need not track it (as CPython untracks such tuples itself; with ~10^5 live records
  // the cyclic collector's passes cost ~70% of a per-record produce)
  if (PyObject_GC_IsTracked(m)) PyObject_GC_UnTrack(m);
  return m;
}

// Every record of a columnar batch as a Message (bytes sliced straight out of the buffers).
py::list build_messages(py::object cls, py::object topic, py::object partition, int64_t base,
                        py::array_t<uint8_t> keys, py::array_t<int64_t> koff, py::array_t<uint8_t> vals,
                        py::array_t<int64_t> voff, py::object null_keys, int64_t ts_ms) {
  const int64_t n = voff.size() - 1;
  const char* kb = reinterpret_cast<const char*>(keys.data());
  const char* vb = reinterpret_cast<const char*>(vals.data());
  const int64_t* ko = koff.data();
  const int64_t* vo = voff.data();
  const uint8_t* nk = nullptr;
  py::array_t<uint8_t> nk_arr;
  if (!null_keys.is_none()) {
    nk_arr = py::array_t<uint8_t>::ensure(null_keys);
    nk = nk_arr.data();
  }
  PyObject* out = PyList_New(n > 0 ? n : 0);
  if (!out) throw py::error_already_set();
  py::object ts = py::reinterpret_steal<py::object>(PyLong_FromLongLong(ts_ms));
  for (int64_t i = 0; i < n; ++i) {
    PyObject* k = (nk && nk[i]) ? (Py_INCREF(Py_None), Py_None) : PyBytes_FromStringAndSize(kb + ko[i], ko[i + 1] - ko[i]);
    PyObject* v = PyBytes_FromStringAndSize(vb + vo[i], vo[i + 1] - vo[i]);
    PyObject* off = PyLong_FromLongLong(base + i);
    Py_INCREF(ts.ptr());
    PyObject* m = (k && v && off) ? new_message(cls.ptr(), topic.ptr(), partition.ptr(), off, k, v, ts.ptr()) : nullptr;
    Py_XDECREF(k);
    Py_XDECREF(v);
    if (!m) {
      Py_XDECREF(off);
      Py_DECREF(ts.ptr());
      Py_DECREF(out);
      throw py::error_already_set();
    }
    PyList_SET_ITEM(out, i, m);
  }
  return py::reinterpret_steal<py::list>(out);
}

// ------------------------------------------------------------------------------------------------
// The in-memory broker's per-record produce in C (stream/fake_kafka.py Producer.produce): the same
// operations on the same Python objects -- under the broker's lock, route by crc32 (zlib's), two
// list appends on the partition's tail, a Message for the delivery report -- without a Python
// frame, as a librdkafka producer would cost. Anything unusual (fault injection, a new topic,
// non-bytes payloads) goes to the Python implementation.
uint32_t crc32_ieee(const uint8_t* p, size_t n) {
  static uint32_t table[256];
  static bool init = false;
  if (!init) {
    for (uint32_t i = 0; i < 256; ++i) {
      uint32_t c = i;
      for (int k = 0; k < 8; ++k) c = (c & 1) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
      table[i] = c;
    }
    init = true;
  }
  uint32_t c = 0xFFFFFFFFu;
  for (size_t i = 0; i < n; ++i) c = table[(c ^ p[i]) & 0xFF] ^ (c >> 8);
  return c ^ 0xFFFFFFFFu;
}

struct FastNames {
  PyObject *lock, *acquire, *release, *topics, *tk, *tv, *tts, *size, *waiting, *cond, *notify_all, *pending,
      *fail_next, *slow, *callback, *partition;
  FastNames() {
    lock = PyUnicode_InternFromString("lock");
    acquire = PyUnicode_InternFromString("acquire");
    release = PyUnicode_InternFromString("release");
    topics = PyUnicode_InternFromString("topics");
    tk = PyUnicode_InternFromString("_tk");
    tv = PyUnicode_InternFromString("_tv");
    tts = PyUnicode_InternFromString("_tts");
    size = PyUnicode_InternFromString("size");
    waiting = PyUnicode_InternFromString("waiting");
    cond = PyUnicode_InternFromString("cond");
    notify_all = PyUnicode_InternFromString("notify_all");
    pending = PyUnicode_InternFromString("_pending");
    fail_next = PyUnicode_InternFromString("fail_next");
    slow = PyUnicode_InternFromString("_produce_py");
    callback = PyUnicode_InternFromString("callback");
    partition = PyUnicode_InternFromString("partition");
  }
};
const FastNames& fnames() {
  static FastNames* n = new FastNames();
  return *n;
}

// state = (producer, broker, Message class, broker.lock.acquire, broker.lock.release, broker.topics)
PyObject* fast_produce(PyObject* state, PyObject* const* args, Py_ssize_t nargs, PyObject* kwnames) {
  const Names& N = names();
  const FastNames& F = fnames();
  PyObject* producer = PyTuple_GET_ITEM(state, 0);
  PyObject* broker = PyTuple_GET_ITEM(state, 1);
  PyObject* cls = PyTuple_GET_ITEM(state, 2);
  PyObject* acquire = PyTuple_GET_ITEM(state, 3);
  PyObject* release = PyTuple_GET_ITEM(state, 4);
  PyObject* topics = PyTuple_GET_ITEM(state, 5);
  PyObject *topic = nargs > 0 ? args[0] : nullptr, *value = nargs > 1 ? args[1] : Py_None,
           *key = nargs > 2 ? args[2] : Py_None, *part_o = nargs > 3 ? args[3] : nullptr, *cb = Py_None;
  bool simple = nargs <= 4;
  const Py_ssize_t nkw = kwnames ? PyTuple_GET_SIZE(kwnames) : 0;
  for (Py_ssize_t i = 0; i < nkw && simple; ++i) {
    PyObject* k = PyTuple_GET_ITEM(kwnames, i);
    PyObject* v = args[nargs + i];
    // interned keyword names compare by identity first
    if (k == N.value || PyUnicode_Compare(k, N.value) == 0) value = v;
    else if (k == N.key || PyUnicode_Compare(k, N.key) == 0) key = v;
    else if (k == N.on_delivery || PyUnicode_Compare(k, N.on_delivery) == 0 || PyUnicode_Compare(k, F.callback) == 0)
      cb = v;
    else if (PyUnicode_Compare(k, F.partition) == 0) part_o = v;
    else simple = false;
  }
  long part = -1;
  if (part_o && part_o != Py_None) {
    part = PyLong_AsLong(part_o);
    if (part == -1 && PyErr_Occurred()) return nullptr;
  }
  PyObject* fail = simple ? PyObject_GetAttr(producer, F.fail_next) : nullptr;
  if (simple && (!fail || PyObject_IsTrue(fail))) simple = false;
  Py_XDECREF(fail);
  PyErr_Clear();
  simple = simple && topic && PyUnicode_Check(topic) && (PyBytes_CheckExact(value) || value == Py_None) &&
           (PyBytes_CheckExact(key) || key == Py_None);
  PyObject* parts = nullptr;
  if (simple) {
    parts = PyDict_GetItemWithError(topics, topic);   // borrowed
    Py_XINCREF(parts);
    if (!parts || !PyList_Check(parts) || PyList_GET_SIZE(parts) == 0) simple = false;
  }
  if (!simple) {                                   // the Python implementation
    Py_XDECREF(parts);
    PyErr_Clear();
    PyObject* slow = PyObject_GetAttr(producer, F.slow);
    if (!slow) return nullptr;
    PyObject* r = PyObject_Vectorcall(slow, args, nargs, kwnames);
    Py_DECREF(slow);
    return r;
  }
  const Py_ssize_t np_ = PyList_GET_SIZE(parts);
  if (part < 0) {
    PyObject* src = key != Py_None && PyBytes_GET_SIZE(key) ? key : value;
    const uint32_t c = src != Py_None ? crc32_ieee(reinterpret_cast<const uint8_t*>(PyBytes_AS_STRING(src)),
                                                   (size_t)PyBytes_GET_SIZE(src))
                                      : 0u;
    part = (long)(c % (uint32_t)np_);
  }
  if (part >= np_) {
    Py_DECREF(parts);
    PyErr_SetString(PyExc_ValueError, "partition out of range");
    return nullptr;
  }
  PyObject* r = PyObject_CallNoArgs(acquire);
  if (!r) {
    Py_DECREF(parts);
    return nullptr;
  }
  Py_DECREF(r);
  PyObject* pobj = PyList_GET_ITEM(parts, part);
  PyObject* tk = PyObject_GetAttr(pobj, F.tk);
  PyObject* tv = PyObject_GetAttr(pobj, F.tv);
  PyObject* size = PyObject_GetAttr(pobj, F.size);
  long long off = -1;
  bool ok = tk && tv && size && PyList_Check(tk) && PyList_Check(tv);
  if (ok && PyList_GET_SIZE(tk) == 0) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);                   // time.perf_counter's clock on Linux
    PyObject* now = PyFloat_FromDouble((double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec);
    ok = now && PyObject_SetAttr(pobj, F.tts, now) == 0;
    Py_XDECREF(now);
  }
  if (ok) ok = PyList_Append(tk, key) == 0 && PyList_Append(tv, value) == 0;
  if (ok) {
    off = PyLong_AsLongLong(size);
    PyObject* ns = PyLong_FromLongLong(off + 1);
    ok = ns && PyObject_SetAttr(pobj, F.size, ns) == 0;
    Py_XDECREF(ns);
  }
  if (ok) {
    PyObject* w = PyObject_GetAttr(broker, F.waiting);
    if (w && PyObject_IsTrue(w)) {
      PyObject* cond = PyObject_GetAttr(broker, F.cond);
      PyObject* rr = cond ? PyObject_CallMethodNoArgs(cond, F.notify_all) : nullptr;
      ok = rr != nullptr;
      Py_XDECREF(rr);
      Py_XDECREF(cond);
    }
    Py_XDECREF(w);
  }
  // release the lock whatever happened (keep a pending error)
  PyObject *et, *ev, *etb;
  PyErr_Fetch(&et, &ev, &etb);
  PyObject* rel = PyObject_CallNoArgs(release);
  Py_XDECREF(rel);
  if (et) PyErr_Restore(et, ev, etb);
  Py_XDECREF(tk);
  Py_XDECREF(tv);
  Py_XDECREF(size);
  Py_DECREF(parts);
  if (!ok || !rel) return nullptr;
  if (cb != Py_None && Py_TYPE(cb) == &DeliveryCounterType) {
    // a DeliveryCounter ignores the report's Message: queue (cb, None, None), no Message built
    PyObject* item = PyTuple_Pack(3, cb, Py_None, Py_None);
    if (item && PyObject_GC_IsTracked(item)) PyObject_GC_UnTrack(item);
    PyObject* pend = item ? PyObject_GetAttr(producer, F.pending) : nullptr;
    const int rc = pend ? PyList_Append(pend, item) : -1;
    Py_XDECREF(pend);
    Py_XDECREF(item);
    if (rc < 0) return nullptr;
  } else if (cb != Py_None) {
    struct timespec ts;
    clock_gettime(CLOCK_REALTIME, &ts);
    PyObject* tms = PyLong_FromLongLong((long long)ts.tv_sec * 1000 + ts.tv_nsec / 1000000);
    PyObject* po = PyLong_FromLong(part);
    PyObject* oo = PyLong_FromLongLong(off);
    PyObject* msg = (tms && po && oo) ? new_message(cls, topic, po, oo, key, value, tms) : nullptr;
    Py_XDECREF(po);
    if (!msg) {
      Py_XDECREF(tms);
      Py_XDECREF(oo);
      return nullptr;
    }
    PyObject* item = PyTuple_Pack(3, cb, Py_None, msg);
    Py_DECREF(msg);
    // a delivery-report entry lives until the next poll, which drops it: untracked like the Message
    if (item && PyObject_GC_IsTracked(item)) PyObject_GC_UnTrack(item);
    PyObject* pend = item ? PyObject_GetAttr(producer, F.pending) : nullptr;
    const int rc = pend ? PyList_Append(pend, item) : -1;
    Py_XDECREF(pend);
    Py_XDECREF(item);
    if (rc < 0) return nullptr;
  }
  Py_RETURN_NONE;
}

// cb(err, what) for every (cb, err, what) of a producer's pending delivery reports, in order
// (the in-memory producer's poll loop, without a bytecode iteration per record)
int64_t deliver_reports(py::list pend) {
  const Py_ssize_t n = PyList_GET_SIZE(pend.ptr());
  for (Py_ssize_t i = 0; i < n; ++i) {
    PyObject* it = PyList_GET_ITEM(pend.ptr(), i);
    if (!PyTuple_Check(it) || PyTuple_GET_SIZE(it) != 3) throw py::type_error("pending report must be (cb, err, what)");
    PyObject* args[2] = {PyTuple_GET_ITEM(it, 1), PyTuple_GET_ITEM(it, 2)};
    PyObject* r = PyObject_Vectorcall(PyTuple_GET_ITEM(it, 0), args, 2, nullptr);
    if (!r) throw py::error_already_set();
    Py_DECREF(r);
  }
  return n;
}

PyMethodDef fast_produce_def = {"produce", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)(void)>(fast_produce)),
                                METH_FASTCALL | METH_KEYWORDS, "in-memory broker produce (C)"};

py::object make_fast_produce(py::object producer, py::object broker, py::object message_cls) {
  py::object lock = broker.attr("lock");
  py::tuple state = py::make_tuple(producer, broker, message_cls, lock.attr("acquire"), lock.attr("release"),
                                   broker.attr("topics"));
  PyObject* f = PyCFunction_NewEx(&fast_produce_def, state.ptr(), nullptr);
  if (!f) throw py::error_already_set();
  return py::reinterpret_steal<py::object>(f);
}

}  // namespace

void register_kafka_ops(pybind11::module& m) {
  m.def("pack_messages", &pack_messages, "consumed Message list -> columnar buffers (C loops)", py::arg("msgs"),
        py::arg("vals_buf") = py::none(), py::arg("by_ref") = false);
  m.def("produce_each", &produce_each, "per-record produce of one output segment from a C loop");
  m.def("install_message_accessors", &install_message_accessors, "C method descriptors on a tuple Message class");
  m.def("build_messages", &build_messages, "columnar batch -> list of Message (C loop)");
  m.def("make_fast_produce", &make_fast_produce, "C produce bound to an in-memory producer");
  m.def("deliver_reports", &deliver_reports, "run (cb, err, what) delivery reports in order (C loop)");
  if (PyType_Ready(&DeliveryCounterType) < 0) throw py::error_already_set();
  Py_INCREF(&DeliveryCounterType);
  m.add_object("DeliveryCounter", py::reinterpret_borrow<py::object>(reinterpret_cast<PyObject*>(&DeliveryCounterType)));
}

// flexmi C API implementation (see flexmi_c.h).  Handles own a strong reference to the Python
// object of the runtime; every entry point takes the GIL, so the API can be used from a C
// program (flexmi_init embeds the interpreter) and from threads of a Python process alike.
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#include <dlfcn.h>

#include <cstring>
#include <string>
#include <vector>

#include "flexmi_c.h"

#define FLEXMI_DEF_HANDLE(name) \
  struct name##_s {             \
    PyObject* o;                \
  };
FLEXMI_DEF_HANDLE(flexmi_config)
FLEXMI_DEF_HANDLE(flexmi_model)
FLEXMI_DEF_HANDLE(flexmi_tensor)
FLEXMI_DEF_HANDLE(flexmi_parameter)
FLEXMI_DEF_HANDLE(flexmi_op)
FLEXMI_DEF_HANDLE(flexmi_optimizer)
FLEXMI_DEF_HANDLE(flexmi_initializer)
FLEXMI_DEF_HANDLE(flexmi_perf_metrics)
FLEXMI_DEF_HANDLE(flexmi_dataloader)
#undef FLEXMI_DEF_HANDLE

namespace {

thread_local std::string g_err;
PyThreadState* g_saved = nullptr;
std::vector<std::string> g_argv;

struct Gil {
  PyGILState_STATE s;
  Gil() : s(PyGILState_Ensure()) {}
  ~Gil() { PyGILState_Release(s); }
};

void capture_error(const char* where) {
  g_err = where;
  if (!PyErr_Occurred()) return;
  PyObject *t, *v, *tb;
  PyErr_Fetch(&t, &v, &tb);
  PyErr_NormalizeException(&t, &v, &tb);
  if (v) {
    PyObject* s = PyObject_Str(v);
    if (s) {
      const char* c = PyUnicode_AsUTF8(s);
      if (c) g_err += std::string(": ") + c;
      Py_DECREF(s);
    }
  }
  PyErr_Restore(t, v, tb);
  PyErr_Print();  // traceback to stderr, clears the error
}

PyObject* import(const char* name) {
  PyObject* m = PyImport_ImportModule(name);
  if (!m) capture_error(name);
  return m;
}

// attribute of a module, new reference
PyObject* attr(const char* mod, const char* name) {
  PyObject* m = import(mod);
  if (!m) return nullptr;
  PyObject* a = PyObject_GetAttrString(m, name);
  Py_DECREF(m);
  if (!a) capture_error(name);
  return a;
}

PyObject* enum_value(const char* enum_name, int v) {
  PyObject* e = attr("flexmi.core.types", enum_name);
  if (!e) return nullptr;
  PyObject* r = PyObject_CallFunction(e, "i", v);
  Py_DECREF(e);
  if (!r) capture_error(enum_name);
  return r;
}

PyObject* str_or_none(const char* s) {
  if (s) return PyUnicode_FromString(s);
  Py_RETURN_NONE;
}

PyObject* obj_or_none(PyObject* o) {
  if (o) {
    Py_INCREF(o);
    return o;
  }
  Py_RETURN_NONE;
}

// call obj.meth(*args, **kw); steals args / kw; returns new ref or null (error captured)
PyObject* call(PyObject* obj, const char* meth, PyObject* args, PyObject* kw = nullptr) {
  PyObject* f = PyObject_GetAttrString(obj, meth);
  PyObject* r = nullptr;
  if (f && args) r = PyObject_Call(f, args, kw);
  Py_XDECREF(f);
  Py_XDECREF(args);
  Py_XDECREF(kw);
  if (!r) capture_error(meth);
  return r;
}

int call_status(PyObject* obj, const char* meth, PyObject* args) {
  PyObject* r = call(obj, meth, args);
  if (!r) return -1;
  Py_DECREF(r);
  return 0;
}

long call_long(PyObject* obj, const char* meth) {
  PyObject* r = call(obj, meth, PyTuple_New(0));
  if (!r) return -1;
  long v = PyLong_AsLong(r);
  Py_DECREF(r);
  return v;
}

long get_long(PyObject* obj, const char* name) {
  PyObject* r = PyObject_GetAttrString(obj, name);
  if (!r) {
    capture_error(name);
    return -1;
  }
  long v = PyLong_AsLong(r);
  Py_DECREF(r);
  return v;
}

template <class H>
H* wrap(PyObject* o) {
  if (!o || o == Py_None) {
    Py_XDECREF(o);
    return nullptr;
  }
  H* h = new H;
  h->o = o;
  return h;
}

template <class H>
void destroy(H* h) {
  if (!h) return;
  Gil g;
  Py_XDECREF(h->o);
  delete h;
}

PyObject* int_list(const int* v, int n) {
  PyObject* l = PyList_New(n);
  for (int i = 0; i < n; ++i) PyList_SET_ITEM(l, i, PyLong_FromLong(v[i]));
  return l;
}

const char* np_dtype(int data_type) {
  switch (data_type) {
    case 40: return "float32";
    case 41: return "float64";
    case 42: return "int32";
    case 43: return "int64";
    case 44: return "bool";
  }
  return nullptr;
}

size_t dtype_size(int data_type) {
  switch (data_type) {
    case 41: case 43: return 8;
    case 44: return 1;
  }
  return 4;
}

// numpy array COPY of a host buffer, shaped
PyObject* np_from(const void* data, size_t nbytes, const char* dtype, PyObject* shape /* stolen, may be null */) {
  PyObject* np = import("numpy");
  if (!np) {
    Py_XDECREF(shape);
    return nullptr;
  }
  PyObject* mv = PyMemoryView_FromMemory((char*)data, (Py_ssize_t)nbytes, PyBUF_READ);
  PyObject* a = call(np, "frombuffer", Py_BuildValue("(Os)", mv, dtype));
  Py_DECREF(mv);
  Py_DECREF(np);
  if (!a) {
    Py_XDECREF(shape);
    return nullptr;
  }
  PyObject* c = call(a, "copy", PyTuple_New(0));
  Py_DECREF(a);
  if (c && shape) {
    PyObject* r = call(c, "reshape", PyTuple_Pack(1, shape));
    Py_DECREF(c);
    c = r;
  }
  Py_XDECREF(shape);
  return c;
}

// copy a numpy array (any shape) into a host buffer as `dtype`; -1 on size mismatch
int np_to(PyObject* arr, void* out, size_t n, const char* dtype) {
  PyObject* np = import("numpy");
  if (!np) return -1;
  PyObject* c = call(np, "ascontiguousarray", Py_BuildValue("(Os)", arr, dtype));
  Py_DECREF(np);
  if (!c) return -1;
  Py_buffer view;
  if (PyObject_GetBuffer(c, &view, PyBUF_C_CONTIGUOUS) != 0) {
    capture_error("buffer");
    Py_DECREF(c);
    return -1;
  }
  int rc = 0;
  if ((size_t)view.len != n * (size_t)view.itemsize) {
    g_err = "size mismatch: tensor has " + std::to_string(view.len / view.itemsize) + " elements";
    rc = -1;
  } else {
    std::memcpy(out, view.buf, view.len);
  }
  PyBuffer_Release(&view);
  Py_DECREF(c);
  return rc;
}

PyObject* executor(flexmi_model_t m) { return call(m->o, "_ex", PyTuple_New(0)); }

flexmi_tensor_t unary(flexmi_model_t m, const char* fn, flexmi_tensor_t x, const char* name) {
  Gil g;
  PyObject* kw = PyDict_New();
  PyObject* n = str_or_none(name);
  PyDict_SetItemString(kw, "name", n);
  Py_DECREF(n);
  return wrap<flexmi_tensor_s>(call(m->o, fn, PyTuple_Pack(1, x->o), kw));
}

flexmi_tensor_t binary(flexmi_model_t m, const char* fn, flexmi_tensor_t x, flexmi_tensor_t y, const char* name) {
  Gil g;
  PyObject* kw = PyDict_New();
  PyObject* n = str_or_none(name);
  PyDict_SetItemString(kw, "name", n);
  Py_DECREF(n);
  return wrap<flexmi_tensor_s>(call(m->o, fn, PyTuple_Pack(2, x->o, y->o), kw));
}

PyObject* kw_name(const char* name) {
  PyObject* kw = PyDict_New();
  PyObject* n = str_or_none(name);
  PyDict_SetItemString(kw, "name", n);
  Py_DECREF(n);
  return kw;
}

std::string lib_root() {
  const char* env = std::getenv("FLEXMI_HOME");
  if (env && *env) return env;
  Dl_info info;
  if (dladdr((void*)&flexmi_init, &info) && info.dli_fname) {
    std::string p = info.dli_fname;  // <root>/flexmi/libflexmi_c.so
    for (int k = 0; k < 2; ++k) {
      auto s = p.find_last_of('/');
      if (s == std::string::npos) return ".";
      p = p.substr(0, s);
    }
    return p;
  }
  return ".";
}

}  // namespace

extern "C" {

// ---------------------------------------------------------------------------------- runtime
int flexmi_init(int argc, char** argv) {
  g_argv.clear();
  for (int i = 0; i < argc; ++i) g_argv.push_back(argv[i]);
  if (g_argv.empty()) g_argv.push_back("flexmi_c");
  if (!Py_IsInitialized()) {
    Py_InitializeEx(0);
    g_saved = PyEval_SaveThread();  // release the GIL; every call re-takes it
  }
  Gil g;
  PyObject* sys = import("sys");
  if (!sys) return -1;
  PyObject* path = PyObject_GetAttrString(sys, "path");
  PyObject* root = PyUnicode_FromString(lib_root().c_str());
  PyList_Insert(path, 0, root);
  Py_DECREF(root);
  Py_DECREF(path);
  PyObject* av = PyList_New(0);
  for (auto& a : g_argv) {
    PyObject* s = PyUnicode_FromString(a.c_str());
    PyList_Append(av, s);
    Py_DECREF(s);
  }
  PyObject_SetAttrString(sys, "argv", av);
  Py_DECREF(av);
  Py_DECREF(sys);
  PyObject* core = import("flexmi.core");
  if (!core) return -1;
  Py_DECREF(core);
  return 0;
}

void flexmi_finalize(void) {
  // The interpreter (and torch's device state) stays alive until process exit; only flush.
  Gil g;
  PyObject* sys = PyImport_ImportModule("sys");
  if (sys) {
    PyObject* out = PyObject_GetAttrString(sys, "stdout");
    if (out) {
      PyObject* r = PyObject_CallMethod(out, "flush", nullptr);
      Py_XDECREF(r);
      Py_DECREF(out);
    }
    Py_DECREF(sys);
  }
  PyErr_Clear();
}

const char* flexmi_last_error(void) { return g_err.c_str(); }

double flexmi_get_current_time(flexmi_config_t c) {
  Gil g;
  PyObject* r = call(c->o, "get_current_time", PyTuple_New(0));
  if (!r) return -1;
  double v = PyFloat_AsDouble(r);
  Py_DECREF(r);
  return v;
}

void flexmi_begin_trace(flexmi_config_t c, int id) {
  Gil g;
  call_status(c->o, "begin_trace", Py_BuildValue("(i)", id));
}

void flexmi_end_trace(flexmi_config_t c, int id) {
  Gil g;
  call_status(c->o, "end_trace", Py_BuildValue("(i)", id));
}

// ---------------------------------------------------------------------------------- config
flexmi_config_t flexmi_config_create(void) {
  Gil g;
  PyObject* cls = attr("flexmi.core", "FFConfig");
  if (!cls) return nullptr;
  PyObject* o = PyObject_CallNoArgs(cls);
  Py_DECREF(cls);
  if (!o) capture_error("FFConfig");
  return wrap<flexmi_config_s>(o);
}

void flexmi_config_destroy(flexmi_config_t c) { destroy(c); }

int flexmi_config_parse_args(flexmi_config_t c, int argc, char** argv) {
  Gil g;
  PyObject* l = PyList_New(0);
  for (int i = 0; i < argc; ++i) {
    PyObject* s = PyUnicode_FromString(argv[i]);
    PyList_Append(l, s);
    Py_DECREF(s);
  }
  int rc = call_status(c->o, "parse_args", PyTuple_Pack(1, l));
  Py_DECREF(l);
  return rc;
}

int flexmi_config_parse_args_default(flexmi_config_t c) {
  std::vector<char*> v;
  for (auto& a : g_argv) v.push_back(const_cast<char*>(a.c_str()));
  return flexmi_config_parse_args(c, (int)v.size(), v.data());
}

int flexmi_config_get_batch_size(flexmi_config_t c) {
  Gil g;
  return (int)get_long(c->o, "batchSize");
}

int flexmi_config_set_batch_size(flexmi_config_t c, int b) {
  Gil g;
  PyObject* v = PyLong_FromLong(b);
  int rc = PyObject_SetAttrString(c->o, "batchSize", v);
  Py_DECREF(v);
  return rc;
}

int flexmi_config_get_workers_per_node(flexmi_config_t c) {
  Gil g;
  return (int)get_long(c->o, "workersPerNode");
}

int flexmi_config_get_num_nodes(flexmi_config_t c) {
  Gil g;
  return (int)get_long(c->o, "numNodes");
}

int flexmi_config_get_epochs(flexmi_config_t c) {
  Gil g;
  return (int)get_long(c->o, "epochs");
}

int flexmi_config_set_device(flexmi_config_t c, const char* device) {
  Gil g;
  PyObject* v = PyUnicode_FromString(device);
  int rc = PyObject_SetAttrString(c->o, "device", v);
  Py_DECREF(v);
  PyObject* a = PyUnicode_FromString("auto");
  rc |= PyObject_SetAttrString(c->o, "compute_dtype", a);
  Py_DECREF(a);
  if (rc == 0) rc = call_status(c->o, "_finalize", PyTuple_New(0));
  return rc;
}

// ---------------------------------------------------------------------------------- model
flexmi_model_t flexmi_model_create(flexmi_config_t c) {
  Gil g;
  PyObject* cls = attr("flexmi.core", "FFModel");
  if (!cls) return nullptr;
  PyObject* o = PyObject_CallOneArg(cls, c->o);
  Py_DECREF(cls);
  if (!o) capture_error("FFModel");
  return wrap<flexmi_model_s>(o);
}

void flexmi_model_destroy(flexmi_model_t m) { destroy(m); }

int flexmi_model_compile(flexmi_model_t m, flexmi_optimizer_t opt, int loss_type, const int* metrics, int n) {
  Gil g;
  PyObject* lt = enum_value("LossType", loss_type);
  if (!lt) return -1;
  PyObject* ml = PyList_New(0);
  for (int i = 0; i < n; ++i) {
    PyObject* e = enum_value("MetricsType", metrics[i]);
    if (!e) {
      Py_DECREF(ml);
      Py_DECREF(lt);
      return -1;
    }
    PyList_Append(ml, e);
    Py_DECREF(e);
  }
  PyObject* o = obj_or_none(opt ? opt->o : nullptr);
  int rc = call_status(m->o, "compile", PyTuple_Pack(3, o, lt, ml));
  Py_DECREF(o);
  Py_DECREF(lt);
  Py_DECREF(ml);
  return rc;
}

#define MODEL_VOID(fn, meth)                                   \
  int fn(flexmi_model_t m) {                                   \
    Gil g;                                                     \
    return call_status(m->o, meth, PyTuple_New(0));            \
  }
MODEL_VOID(flexmi_model_init_layers, "init_layers")
MODEL_VOID(flexmi_model_forward, "forward")
MODEL_VOID(flexmi_model_backward, "backward")
MODEL_VOID(flexmi_model_update, "update")
MODEL_VOID(flexmi_model_zero_gradients, "zero_gradients")
MODEL_VOID(flexmi_model_reset_metrics, "reset_metrics")
MODEL_VOID(flexmi_model_compute_metrics, "compute_metrics")
MODEL_VOID(flexmi_model_prefetch, "prefetch")
#undef MODEL_VOID

int flexmi_model_print_layers(flexmi_model_t m, int id) {
  Gil g;
  return call_status(m->o, "print_layers", Py_BuildValue("(i)", id));
}

int flexmi_model_set_sgd_optimizer(flexmi_model_t m, flexmi_optimizer_t o) {
  Gil g;
  return call_status(m->o, "set_sgd_optimizer", PyTuple_Pack(1, o->o));
}

int flexmi_model_set_adam_optimizer(flexmi_model_t m, flexmi_optimizer_t o) {
  Gil g;
  return call_status(m->o, "set_adam_optimizer", PyTuple_Pack(1, o->o));
}

flexmi_tensor_t flexmi_model_get_label_tensor(flexmi_model_t m) {
  Gil g;
  return wrap<flexmi_tensor_s>(call(m->o, "get_label_tensor", PyTuple_New(0)));
}

flexmi_op_t flexmi_model_get_layer_by_id(flexmi_model_t m, int id) {
  Gil g;
  return wrap<flexmi_op_s>(call(m->o, "get_layer_by_id", Py_BuildValue("(i)", id)));
}

flexmi_parameter_t flexmi_model_get_parameter_by_id(flexmi_model_t m, int id) {
  Gil g;
  return wrap<flexmi_parameter_s>(call(m->o, "get_parameter_by_id", Py_BuildValue("(i)", id)));
}

flexmi_perf_metrics_t flexmi_model_get_perf_metrics(flexmi_model_t m) {
  Gil g;
  return wrap<flexmi_perf_metrics_s>(call(m->o, "get_perf_metrics", PyTuple_New(0)));
}

int flexmi_model_save_checkpoint(flexmi_model_t m, const char* path) {
  Gil g;
  return call_status(m->o, "save_checkpoint", Py_BuildValue("(s)", path));
}

int flexmi_model_load_checkpoint(flexmi_model_t m, const char* path) {
  Gil g;
  return call_status(m->o, "load_checkpoint", Py_BuildValue("(s)", path));
}

// ---------------------------------------------------------------------------------- builders
flexmi_tensor_t flexmi_tensor_create(flexmi_model_t m, int ndims, const int* dims, int data_type, int create_grad,
                                     const char* name) {
  Gil g;
  PyObject* dt = enum_value("DataType", data_type);
  if (!dt) return nullptr;
  PyObject* kw = kw_name(name);
  PyObject* cg = PyBool_FromLong(create_grad);
  PyDict_SetItemString(kw, "create_grad", cg);
  Py_DECREF(cg);
  PyObject* r = call(m->o, "create_tensor", Py_BuildValue("(NN)", int_list(dims, ndims), dt), kw);
  return wrap<flexmi_tensor_s>(r);
}

flexmi_tensor_t flexmi_model_add_exp(flexmi_model_t m, flexmi_tensor_t x, const char* n) { return unary(m, "exp", x, n); }
flexmi_tensor_t flexmi_model_add_relu(flexmi_model_t m, flexmi_tensor_t x, const char* n) { return unary(m, "relu", x, n); }
flexmi_tensor_t flexmi_model_add_sigmoid(flexmi_model_t m, flexmi_tensor_t x, const char* n) {
  return unary(m, "sigmoid", x, n);
}
flexmi_tensor_t flexmi_model_add_tanh(flexmi_model_t m, flexmi_tensor_t x, const char* n) { return unary(m, "tanh", x, n); }
flexmi_tensor_t flexmi_model_add_elu(flexmi_model_t m, flexmi_tensor_t x, const char* n) { return unary(m, "elu", x, n); }
flexmi_tensor_t flexmi_model_add_flat(flexmi_model_t m, flexmi_tensor_t x, const char* n) { return unary(m, "flat", x, n); }
flexmi_tensor_t flexmi_model_add_softmax(flexmi_model_t m, flexmi_tensor_t x, const char* n) {
  return unary(m, "softmax", x, n);
}
flexmi_tensor_t flexmi_model_add_add(flexmi_model_t m, flexmi_tensor_t x, flexmi_tensor_t y, const char* n) {
  return binary(m, "add", x, y, n);
}
flexmi_tensor_t flexmi_model_add_subtract(flexmi_model_t m, flexmi_tensor_t x, flexmi_tensor_t y, const char* n) {
  return binary(m, "subtract", x, y, n);
}
flexmi_tensor_t flexmi_model_add_multiply(flexmi_model_t m, flexmi_tensor_t x, flexmi_tensor_t y, const char* n) {
  return binary(m, "multiply", x, y, n);
}
flexmi_tensor_t flexmi_model_add_divide(flexmi_model_t m, flexmi_tensor_t x, flexmi_tensor_t y, const char* n) {
  return binary(m, "divide", x, y, n);
}
flexmi_tensor_t flexmi_model_add_batch_matmul(flexmi_model_t m, flexmi_tensor_t a, flexmi_tensor_t b, const char* n) {
  return binary(m, "batch_matmul", a, b, n);
}

flexmi_tensor_t flexmi_model_add_conv2d(flexmi_model_t m, flexmi_tensor_t x, int oc, int kh, int kw_, int sh, int sw,
                                        int ph, int pw, int act, int use_bias, flexmi_initializer_t ki,
                                        flexmi_initializer_t bi, const char* name) {
  Gil g;
  PyObject* a = enum_value("ActiMode", act);
  if (!a) return nullptr;
  PyObject* kw = kw_name(name);
  PyDict_SetItemString(kw, "use_bias", use_bias ? Py_True : Py_False);
  if (ki) PyDict_SetItemString(kw, "kernel_initializer", ki->o);
  if (bi) PyDict_SetItemString(kw, "bias_initializer", bi->o);
  return wrap<flexmi_tensor_s>(
      call(m->o, "conv2d", Py_BuildValue("(OiiiiiiiN)", x->o, oc, kh, kw_, sh, sw, ph, pw, a), kw));
}

flexmi_tensor_t flexmi_model_add_embedding(flexmi_model_t m, flexmi_tensor_t x, int num_entries, int out_dim, int aggr,
                                           flexmi_initializer_t ki, const char* name) {
  Gil g;
  PyObject* a = enum_value("AggrMode", aggr);
  if (!a) return nullptr;
  PyObject* kw = kw_name(name);
  if (ki) PyDict_SetItemString(kw, "kernel_initializer", ki->o);
  return wrap<flexmi_tensor_s>(call(m->o, "embedding", Py_BuildValue("(OiiN)", x->o, num_entries, out_dim, a), kw));
}

flexmi_tensor_t flexmi_model_add_pool2d(flexmi_model_t m, flexmi_tensor_t x, int kh, int kw_, int sh, int sw, int ph,
                                        int pw, int pool_type, int act, const char* name) {
  Gil g;
  PyObject* pt = enum_value("PoolType", pool_type);
  PyObject* a = enum_value("ActiMode", act);
  if (!pt || !a) {
    Py_XDECREF(pt);
    Py_XDECREF(a);
    return nullptr;
  }
  return wrap<flexmi_tensor_s>(
      call(m->o, "pool2d", Py_BuildValue("(OiiiiiiNN)", x->o, kh, kw_, sh, sw, ph, pw, pt, a), kw_name(name)));
}

flexmi_tensor_t flexmi_model_add_batch_norm(flexmi_model_t m, flexmi_tensor_t x, int relu, const char* name) {
  Gil g;
  return wrap<flexmi_tensor_s>(
      call(m->o, "batch_norm", Py_BuildValue("(OO)", x->o, relu ? Py_True : Py_False), kw_name(name)));
}

flexmi_tensor_t flexmi_model_add_dense(flexmi_model_t m, flexmi_tensor_t x, int out_dim, int act, int use_bias,
                                       flexmi_initializer_t ki, flexmi_initializer_t bi, const char* name) {
  Gil g;
  PyObject* a = enum_value("ActiMode", act);
  if (!a) return nullptr;
  PyObject* kw = kw_name(name);
  PyDict_SetItemString(kw, "use_bias", use_bias ? Py_True : Py_False);
  if (ki) PyDict_SetItemString(kw, "kernel_initializer", ki->o);
  if (bi) PyDict_SetItemString(kw, "bias_initializer", bi->o);
  return wrap<flexmi_tensor_s>(call(m->o, "dense", Py_BuildValue("(OiN)", x->o, out_dim, a), kw));
}

flexmi_tensor_t flexmi_model_add_concat(flexmi_model_t m, int n, const flexmi_tensor_t* xs, int axis,
                                        const char* name) {
  Gil g;
  PyObject* l = PyList_New(n);
  for (int i = 0; i < n; ++i) {
    Py_INCREF(xs[i]->o);
    PyList_SET_ITEM(l, i, xs[i]->o);
  }
  return wrap<flexmi_tensor_s>(call(m->o, "concat", Py_BuildValue("(Ni)", l, axis), kw_name(name)));
}

int flexmi_model_add_split(flexmi_model_t m, flexmi_tensor_t x, int n, const int* sizes, int axis,
                           flexmi_tensor_t* outputs, const char* name) {
  Gil g;
  PyObject* r = call(m->o, "split", Py_BuildValue("(ONi)", x->o, int_list(sizes, n), axis), kw_name(name));
  if (!r) return -1;
  PyObject* seq = PySequence_Fast(r, "split result");
  Py_DECREF(r);
  if (!seq) {
    capture_error("split");
    return -1;
  }
  Py_ssize_t k = PySequence_Fast_GET_SIZE(seq);
  for (Py_ssize_t i = 0; i < k && i < n; ++i) {
    PyObject* t = PySequence_Fast_GET_ITEM(seq, i);
    Py_INCREF(t);
    outputs[i] = wrap<flexmi_tensor_s>(t);
  }
  Py_DECREF(seq);
  return (int)k;
}

flexmi_tensor_t flexmi_model_add_reshape(flexmi_model_t m, flexmi_tensor_t x, int nd, const int* shape,
                                         const char* name) {
  Gil g;
  return wrap<flexmi_tensor_s>(call(m->o, "reshape", Py_BuildValue("(ON)", x->o, int_list(shape, nd)), kw_name(name)));
}

flexmi_tensor_t flexmi_model_add_transpose(flexmi_model_t m, flexmi_tensor_t x, int nd, const int* perm,
                                           const char* name) {
  Gil g;
  return wrap<flexmi_tensor_s>(call(m->o, "transpose", Py_BuildValue("(ON)", x->o, int_list(perm, nd)), kw_name(name)));
}

flexmi_tensor_t flexmi_model_add_reverse(flexmi_model_t m, flexmi_tensor_t x, int axis, const char* name) {
  Gil g;
  return wrap<flexmi_tensor_s>(call(m->o, "reverse", Py_BuildValue("(Oi)", x->o, axis), kw_name(name)));
}

flexmi_tensor_t flexmi_model_add_dropout(flexmi_model_t m, flexmi_tensor_t x, float rate, unsigned long long seed,
                                         const char* name) {
  Gil g;
  return wrap<flexmi_tensor_s>(call(m->o, "dropout", Py_BuildValue("(OdK)", x->o, (double)rate, seed), kw_name(name)));
}

// ---------------------------------------------------------------------------------- tensors
void flexmi_tensor_destroy(flexmi_tensor_t t) { destroy(t); }

int flexmi_tensor_get_num_dims(flexmi_tensor_t t) {
  Gil g;
  return (int)get_long(t->o, "num_dims");
}

int flexmi_tensor_get_dims(flexmi_tensor_t t, int* dims) {
  Gil g;
  PyObject* d = PyObject_GetAttrString(t->o, "dims");
  if (!d) {
    capture_error("dims");
    return -1;
  }
  Py_ssize_t n = PySequence_Size(d);
  for (Py_ssize_t i = 0; i < n; ++i) {
    PyObject* v = PySequence_GetItem(d, i);
    dims[i] = (int)PyLong_AsLong(v);
    Py_DECREF(v);
  }
  Py_DECREF(d);
  return (int)n;
}

int flexmi_tensor_get_data_type(flexmi_tensor_t t) {
  Gil g;
  PyObject* d = PyObject_GetAttrString(t->o, "data_type");
  if (!d) {
    capture_error("data_type");
    return -1;
  }
  long v = PyLong_AsLong(d);
  Py_DECREF(d);
  return (int)v;
}

flexmi_op_t flexmi_tensor_get_owner_op(flexmi_tensor_t t) {
  Gil g;
  return wrap<flexmi_op_s>(PyObject_GetAttrString(t->o, "owner_op"));
}

static int set_array(flexmi_model_t m, flexmi_tensor_t t, const void* data, size_t n, size_t es, const char* dtype) {
  Gil g;
  PyObject* ex = executor(m);
  if (!ex) return -1;
  PyObject* a = np_from(data, n * es, dtype, nullptr);
  if (!a) {
    Py_DECREF(ex);
    return -1;
  }
  int rc = call_status(ex, "scatter_from_host", PyTuple_Pack(2, t->o, a));
  Py_DECREF(a);
  Py_DECREF(ex);
  return rc;
}

int flexmi_tensor_set_array_float(flexmi_model_t m, flexmi_tensor_t t, const float* d, size_t n) {
  return set_array(m, t, d, n, 4, "float32");
}
int flexmi_tensor_set_array_int32(flexmi_model_t m, flexmi_tensor_t t, const int32_t* d, size_t n) {
  return set_array(m, t, d, n, 4, "int32");
}
int flexmi_tensor_set_array_int64(flexmi_model_t m, flexmi_tensor_t t, const int64_t* d, size_t n) {
  return set_array(m, t, d, n, 8, "int64");
}

int flexmi_tensor_get_array_float(flexmi_model_t m, flexmi_tensor_t t, float* out, size_t n) {
  Gil g;
  PyObject* ex = executor(m);
  if (!ex) return -1;
  PyObject* a = call(ex, "gather_to_host", PyTuple_Pack(1, t->o));
  Py_DECREF(ex);
  if (!a) return -1;
  int rc = np_to(a, out, n, "float32");
  Py_DECREF(a);
  return rc;
}

// ---------------------------------------------------------------------------------- parameters / ops
void flexmi_parameter_destroy(flexmi_parameter_t p) { destroy(p); }

int flexmi_parameter_get_num_elements(flexmi_parameter_t p) {
  Gil g;
  return (int)call_long(p->o, "volume");
}

int flexmi_parameter_get_weights_float(flexmi_parameter_t p, flexmi_model_t m, float* out, size_t n) {
  Gil g;
  PyObject* a = call(p->o, "get_weights", PyTuple_Pack(1, m->o));
  if (!a) return -1;
  int rc = np_to(a, out, n, "float32");
  Py_DECREF(a);
  return rc;
}

int flexmi_parameter_set_weights_float(flexmi_parameter_t p, flexmi_model_t m, const float* data, size_t n) {
  Gil g;
  PyObject* dims = PyObject_GetAttrString(p->o, "dims");
  if (!dims) {
    capture_error("dims");
    return -1;
  }
  PyObject* shape = PySequence_Tuple(dims);
  Py_DECREF(dims);
  PyObject* a = np_from(data, n * 4, "float32", shape);
  if (!a) return -1;
  int rc = call_status(p->o, "set_weights", PyTuple_Pack(2, m->o, a));
  Py_DECREF(a);
  return rc;
}

void flexmi_op_destroy(flexmi_op_t op) { destroy(op); }

static PyObject* list_item(PyObject* o, const char* attr_name, int id) {
  PyObject* l = PyObject_GetAttrString(o, attr_name);
  if (!l) {
    capture_error(attr_name);
    return nullptr;
  }
  PyObject* r = PySequence_GetItem(l, id);
  Py_DECREF(l);
  if (!r) capture_error(attr_name);
  return r;
}

flexmi_parameter_t flexmi_op_get_parameter_by_id(flexmi_op_t op, int id) {
  Gil g;
  return wrap<flexmi_parameter_s>(list_item(op->o, "weights", id));
}

flexmi_tensor_t flexmi_op_get_input_by_id(flexmi_op_t op, int id) {
  Gil g;
  return wrap<flexmi_tensor_s>(list_item(op->o, "inputs", id));
}

flexmi_tensor_t flexmi_op_get_output_by_id(flexmi_op_t op, int id) {
  Gil g;
  return wrap<flexmi_tensor_s>(list_item(op->o, "outputs", id));
}

int flexmi_op_get_name(flexmi_op_t op, char* buf, size_t len) {
  Gil g;
  PyObject* n = PyObject_GetAttrString(op->o, "name");
  if (!n) {
    capture_error("name");
    return -1;
  }
  const char* s = PyUnicode_AsUTF8(n);
  int rc = s ? (int)std::strlen(s) : -1;
  if (s && len) {
    std::strncpy(buf, s, len - 1);
    buf[len - 1] = 0;
  }
  Py_DECREF(n);
  return rc;
}

// ---------------------------------------------------------------------------------- optimizers etc.
flexmi_optimizer_t flexmi_sgd_optimizer_create(flexmi_model_t m, double lr, double momentum, int nesterov, double wd) {
  Gil g;
  PyObject* cls = attr("flexmi.core", "SGDOptimizer");
  if (!cls) return nullptr;
  PyObject* o = PyObject_Call(cls, Py_BuildValue("(OddOd)", m->o, lr, momentum, nesterov ? Py_True : Py_False, wd),
                              nullptr);
  Py_DECREF(cls);
  if (!o) capture_error("SGDOptimizer");
  return wrap<flexmi_optimizer_s>(o);
}

flexmi_optimizer_t flexmi_adam_optimizer_create(flexmi_model_t m, double alpha, double b1, double b2, double wd,
                                                double eps) {
  Gil g;
  PyObject* cls = attr("flexmi.core", "AdamOptimizer");
  if (!cls) return nullptr;
  PyObject* o = PyObject_Call(cls, Py_BuildValue("(Oddddd)", m->o, alpha, b1, b2, wd, eps), nullptr);
  Py_DECREF(cls);
  if (!o) capture_error("AdamOptimizer");
  return wrap<flexmi_optimizer_s>(o);
}

int flexmi_optimizer_set_lr(flexmi_optimizer_t o, double lr) {
  Gil g;
  return call_status(o->o, "set_learning_rate", Py_BuildValue("(d)", lr));
}

void flexmi_optimizer_destroy(flexmi_optimizer_t o) { destroy(o); }

static flexmi_initializer_t make_init(const char* cls_name, PyObject* args) {
  Gil g;
  PyObject* cls = attr("flexmi.core", cls_name);
  if (!cls) {
    Py_XDECREF(args);
    return nullptr;
  }
  PyObject* o = PyObject_Call(cls, args, nullptr);
  Py_DECREF(cls);
  Py_XDECREF(args);
  if (!o) capture_error(cls_name);
  return wrap<flexmi_initializer_s>(o);
}

flexmi_initializer_t flexmi_glorot_uniform_initializer_create(int seed) {
  Gil g;
  return make_init("GlorotUniformInitializer", Py_BuildValue("(i)", seed));
}
flexmi_initializer_t flexmi_zero_initializer_create(void) {
  Gil g;
  return make_init("ZeroInitializer", PyTuple_New(0));
}
flexmi_initializer_t flexmi_uniform_initializer_create(int seed, float lo, float hi) {
  Gil g;
  return make_init("UniformInitializer", Py_BuildValue("(idd)", seed, (double)lo, (double)hi));
}
flexmi_initializer_t flexmi_norm_initializer_create(int seed, float mean, float std) {
  Gil g;
  return make_init("NormInitializer", Py_BuildValue("(idd)", seed, (double)mean, (double)std));
}
void flexmi_initializer_destroy(flexmi_initializer_t i) { destroy(i); }

static float pm_float(flexmi_perf_metrics_t pm, const char* meth) {
  Gil g;
  PyObject* r = call(pm->o, meth, PyTuple_New(0));
  if (!r) return -1.f;
  float v = (float)PyFloat_AsDouble(r);
  Py_DECREF(r);
  return v;
}
float flexmi_perf_metrics_get_accuracy(flexmi_perf_metrics_t pm) { return pm_float(pm, "get_accuracy"); }
float flexmi_perf_metrics_get_loss(flexmi_perf_metrics_t pm) { return pm_float(pm, "get_loss"); }
void flexmi_perf_metrics_destroy(flexmi_perf_metrics_t pm) { destroy(pm); }

// ---------------------------------------------------------------------------------- data loaders
flexmi_dataloader_t flexmi_single_dataloader_create(flexmi_model_t m, flexmi_tensor_t t, const void* data,
                                                    int num_samples, int data_type) {
  Gil g;
  const char* dt = np_dtype(data_type);
  if (!dt) {
    g_err = "unsupported data type";
    return nullptr;
  }
  PyObject* d = PyObject_GetAttrString(t->o, "dims");
  if (!d) {
    capture_error("dims");
    return nullptr;
  }
  Py_ssize_t nd = PySequence_Size(d);
  size_t per = 1;
  PyObject* shape = PyTuple_New(nd);
  PyTuple_SET_ITEM(shape, 0, PyLong_FromLong(num_samples));
  for (Py_ssize_t i = 1; i < nd; ++i) {
    PyObject* v = PySequence_GetItem(d, i);
    per *= (size_t)PyLong_AsLong(v);
    PyTuple_SET_ITEM(shape, i, v);
  }
  Py_DECREF(d);
  PyObject* arr = np_from(data, per * (size_t)num_samples * dtype_size(data_type), dt, shape);
  if (!arr) return nullptr;
  PyObject* cls = attr("flexmi.core", "SingleDataLoader");
  if (!cls) {
    Py_DECREF(arr);
    return nullptr;
  }
  PyObject* o = PyObject_Call(cls, Py_BuildValue("(OONi)", m->o, t->o, arr, num_samples), nullptr);
  Py_DECREF(cls);
  if (!o) capture_error("SingleDataLoader");
  return wrap<flexmi_dataloader_s>(o);
}

int flexmi_dataloader_next_batch(flexmi_dataloader_t d, flexmi_model_t m) {
  Gil g;
  return call_status(d->o, "next_batch", PyTuple_Pack(1, m->o));
}

int flexmi_dataloader_reset(flexmi_dataloader_t d) {
  Gil g;
  return call_status(d->o, "reset", PyTuple_New(0));
}

int flexmi_dataloader_get_num_samples(flexmi_dataloader_t d) {
  Gil g;
  return (int)call_long(d->o, "get_num_samples");
}

int flexmi_dataloader_set_num_samples(flexmi_dataloader_t d, int n) {
  Gil g;
  return call_status(d->o, "set_num_samples", Py_BuildValue("(i)", n));
}

void flexmi_dataloader_destroy(flexmi_dataloader_t d) { destroy(d); }

// ---------------------------------------------------------------------------------- reference-name parity
void flexmi_sgd_optimizer_destroy(flexmi_optimizer_t o) { flexmi_optimizer_destroy(o); }
int flexmi_sgd_optimizer_set_lr(flexmi_optimizer_t o, double lr) { return flexmi_optimizer_set_lr(o, lr); }
void flexmi_adam_optimizer_destroy(flexmi_optimizer_t o) { flexmi_optimizer_destroy(o); }
int flexmi_adam_optimizer_set_lr(flexmi_optimizer_t o, double lr) { return flexmi_optimizer_set_lr(o, lr); }
flexmi_initializer_t flexmi_initializer_create_null(void) {
  Gil g;
  Py_INCREF(Py_None);
  return wrap<flexmi_initializer_s>(Py_None);
}
void flexmi_glorot_uniform_initializer_destroy(flexmi_initializer_t i) { flexmi_initializer_destroy(i); }
void flexmi_zero_initializer_destroy(flexmi_initializer_t i) { flexmi_initializer_destroy(i); }
void flexmi_uniform_initializer_destroy(flexmi_initializer_t i) { flexmi_initializer_destroy(i); }
void flexmi_norm_initializer_destroy(flexmi_initializer_t i) { flexmi_initializer_destroy(i); }
float flexmi_per_metrics_get_accuracy(flexmi_per_metrics_t pm) { return flexmi_perf_metrics_get_accuracy(pm); }
void flexmi_per_metrics_destroy(flexmi_per_metrics_t pm) { flexmi_perf_metrics_destroy(pm); }

flexmi_tensor_t flexmi_constant_create(flexmi_model_t m, int num_dims, const int* dims, float value, int data_type) {
  Gil g;
  PyObject* dt = enum_value("DataType", data_type);
  if (!dt) return nullptr;
  return wrap<flexmi_tensor_s>(
      call(m->o, "create_constant", Py_BuildValue("(NdN)", int_list(dims, num_dims), (double)value, dt)));
}

static PyObject* init_or_none(flexmi_initializer_t i) { return obj_or_none(i ? i->o : nullptr); }

flexmi_op_t flexmi_model_add_conv2d_no_inout(flexmi_model_t m, int in_channels, int out_channels, int kh, int kw, int sh,
                                             int sw, int ph, int pw, int act, int use_bias, flexmi_initializer_t ki,
                                             flexmi_initializer_t bi) {
  Gil g;
  PyObject* a = enum_value("ActiMode", act);
  if (!a) return nullptr;
  // functional form conv2d(in_c, out_c, kh, kw, sh, sw, ph, pw, act, use_bias, kernel_init, bias_init)
  return wrap<flexmi_op_s>(call(m->o, "conv2d",
                                Py_BuildValue("(iiiiiiiiNONN)", in_channels, out_channels, kh, kw, sh, sw, ph, pw, a,
                                              use_bias ? Py_True : Py_False, init_or_none(ki), init_or_none(bi))));
}

flexmi_op_t flexmi_model_add_pool2d_no_inout(flexmi_model_t m, int kh, int kw, int sh, int sw, int ph, int pw,
                                             int pool_type, int act) {
  Gil g;
  PyObject* pt = enum_value("PoolType", pool_type);
  PyObject* a = enum_value("ActiMode", act);
  if (!pt || !a) {
    Py_XDECREF(pt);
    Py_XDECREF(a);
    return nullptr;
  }
  // functional form pool2d(kh, kw, sh, sw, ph, pw, type, act)
  return wrap<flexmi_op_s>(call(m->o, "pool2d", Py_BuildValue("(iiiiiiNN)", kh, kw, sh, sw, ph, pw, pt, a)));
}

flexmi_op_t flexmi_model_add_dense_no_inout(flexmi_model_t m, int in_dim, int out_dim, int act, int use_bias,
                                            flexmi_initializer_t ki, flexmi_initializer_t bi) {
  Gil g;
  PyObject* a = enum_value("ActiMode", act);
  if (!a) return nullptr;
  // functional form dense(in_dim, out_dim, act, use_bias, kernel_init, bias_init)
  return wrap<flexmi_op_s>(call(m->o, "dense", Py_BuildValue("(iiNONN)", in_dim, out_dim, a, use_bias ? Py_True : Py_False,
                                                             init_or_none(ki), init_or_none(bi))));
}

flexmi_op_t flexmi_model_add_flat_no_inout(flexmi_model_t m) {
  Gil g;
  return wrap<flexmi_op_s>(call(m->o, "flat", PyTuple_New(0)));
}

flexmi_tensor_t flexmi_op_init_inout(flexmi_op_t op, flexmi_model_t m, flexmi_tensor_t input) {
  Gil g;
  return wrap<flexmi_tensor_s>(call(op->o, "init_inout", PyTuple_Pack(2, m->o, input->o)));
}

int flexmi_op_init(flexmi_op_t op, flexmi_model_t m) {
  Gil g;
  return call_status(op->o, "init", PyTuple_Pack(1, m->o));
}

int flexmi_op_forward(flexmi_op_t op, flexmi_model_t m) {
  Gil g;
  return call_status(m->o, "forward_op", PyTuple_Pack(1, op->o));
}

static PyObject* cfg_or_none(flexmi_config_t c) { return obj_or_none(c ? c->o : nullptr); }

int flexmi_tensor_inline_map(flexmi_tensor_t t, flexmi_config_t c) {
  Gil g;
  return call_status(t->o, "inline_map", Py_BuildValue("(N)", cfg_or_none(c)));
}

int flexmi_tensor_inline_unmap(flexmi_tensor_t t, flexmi_config_t c) {
  Gil g;
  return call_status(t->o, "inline_unmap", Py_BuildValue("(N)", cfg_or_none(c)));
}

int flexmi_tensor_is_mapped(flexmi_tensor_t t) {
  Gil g;
  PyObject* r = call(t->o, "is_mapped", PyTuple_New(0));
  if (!r) return -1;
  int v = PyObject_IsTrue(r);
  Py_DECREF(r);
  return v;
}

static void* raw_ptr(flexmi_tensor_t t) {
  Gil g;
  // mapped host array first (the reference returned the mapped region's pointer)
  PyObject* mp = PyObject_GetAttrString(t->o, "_mapped");
  if (mp && mp != Py_None) {
    PyObject* ct = PyObject_GetAttrString(mp, "ctypes");
    PyObject* d = ct ? PyObject_GetAttrString(ct, "data") : nullptr;
    void* p = d ? PyLong_AsVoidPtr(d) : nullptr;
    Py_XDECREF(d);
    Py_XDECREF(ct);
    Py_DECREF(mp);
    if (!p) capture_error("mapped pointer");
    return p;
  }
  Py_XDECREF(mp);
  PyErr_Clear();
  PyObject* r = call(t->o, "get_raw_ptr", PyTuple_New(0));
  if (!r) return nullptr;
  void* p = PyLong_AsVoidPtr(r);
  Py_DECREF(r);
  return p;
}

float* flexmi_tensor_get_raw_ptr_float(flexmi_tensor_t t, flexmi_config_t) { return (float*)raw_ptr(t); }
int32_t* flexmi_tensor_get_raw_ptr_int32(flexmi_tensor_t t, flexmi_config_t) { return (int32_t*)raw_ptr(t); }

int flexmi_tensor_attach_raw_ptr(flexmi_tensor_t t, flexmi_config_t, void* ptr, int column_major) {
  Gil g;
  PyObject* model = PyObject_GetAttrString(t->o, "model");
  if (!model) {
    capture_error("model");
    return -1;
  }
  int rc = call_status(t->o, "attach_raw_ptr",
                       Py_BuildValue("(NNO)", model, PyLong_FromVoidPtr(ptr), column_major ? Py_True : Py_False));
  return rc;
}

int flexmi_tensor_detach_raw_ptr(flexmi_tensor_t t, flexmi_config_t) {
  Gil g;
  return call_status(t->o, "detach_raw_ptr", PyTuple_New(0));
}

struct flexmi_net_config_s {
  std::string dataset_path;
};

flexmi_net_config_t flexmi_net_config_create(void) {
  auto* n = new flexmi_net_config_s();
  for (size_t i = 0; i + 1 < g_argv.size(); ++i)
    if (g_argv[i] == "--dataset" || g_argv[i] == "-d") n->dataset_path = g_argv[i + 1];
  return n;
}
void flexmi_net_config_destroy(flexmi_net_config_t n) { delete n; }
const char* flexmi_net_config_get_dataset_path(flexmi_net_config_t n) { return n ? n->dataset_path.c_str() : ""; }

static flexmi_dataloader_t make_pair_loader(flexmi_model_t m, flexmi_tensor_t input, flexmi_tensor_t label, PyObject* fi,
                                            PyObject* fl, int num_samples) {
  PyObject* cls = attr("flexmi.core", "DataLoader2D");
  if (!cls) {
    Py_XDECREF(fi);
    Py_XDECREF(fl);
    return nullptr;
  }
  PyObject* o = PyObject_Call(cls, Py_BuildValue("(OOOONi)", m->o, input->o, label->o, fi, fl, num_samples), nullptr);
  Py_DECREF(cls);
  if (!o) capture_error("DataLoader2D");
  return wrap<flexmi_dataloader_s>(o);
}

flexmi_dataloader_4d_t flexmi_dataloader_4d_create(flexmi_model_t m, flexmi_net_config_t n, flexmi_tensor_t input,
                                                   flexmi_tensor_t label) {
  Gil g;
  if (n && !n->dataset_path.empty()) {
    g_err = "dataloader_4d_create: dataset files are read by the HDF5 / PrefetchLoader paths (flexmi.models.dlrm)";
    return nullptr;
  }
  // random synthetic data: 4 batches, uniform inputs, integer labels in [0, 10) (float labels uniform)
  PyObject* mod = import("flexmi.core.dataloader");
  if (!mod) return nullptr;
  PyObject* r = call(mod, "synthetic_pair", PyTuple_Pack(3, m->o, input->o, label->o));
  Py_DECREF(mod);
  if (!r) return nullptr;
  PyObject* fi = PyTuple_GetItem(r, 0);
  PyObject* fl = PyTuple_GetItem(r, 1);
  long ns = PyLong_AsLong(PyTuple_GetItem(r, 2));
  Py_INCREF(fi);
  Py_INCREF(fl);
  Py_DECREF(r);
  return make_pair_loader(m, input, label, fi, fl, (int)ns);
}

static PyObject* host_array(flexmi_tensor_t t) {
  PyObject* a = call(t->o, "get_array", PyTuple_New(0));
  return a;
}

flexmi_dataloader_4d_t flexmi_dataloader_4d_create_v2(flexmi_model_t m, flexmi_tensor_t input, flexmi_tensor_t label,
                                                      flexmi_tensor_t full_input, flexmi_tensor_t full_label,
                                                      int num_samples) {
  Gil g;
  PyObject* fi = host_array(full_input);
  PyObject* fl = fi ? host_array(full_label) : nullptr;
  if (!fi || !fl) {
    Py_XDECREF(fi);
    return nullptr;
  }
  return make_pair_loader(m, input, label, fi, fl, num_samples);
}

flexmi_dataloader_2d_t flexmi_dataloader_2d_create_v2(flexmi_model_t m, flexmi_tensor_t input, flexmi_tensor_t label,
                                                      flexmi_tensor_t full_input, flexmi_tensor_t full_label,
                                                      int num_samples) {
  return flexmi_dataloader_4d_create_v2(m, input, label, full_input, full_label, num_samples);
}

int flexmi_dataloader_4d_next_batch(flexmi_dataloader_4d_t d, flexmi_model_t m) { return flexmi_dataloader_next_batch(d, m); }
int flexmi_dataloader_4d_reset(flexmi_dataloader_4d_t d) { return flexmi_dataloader_reset(d); }
int flexmi_dataloader_4d_get_num_samples(flexmi_dataloader_4d_t d) { return flexmi_dataloader_get_num_samples(d); }
int flexmi_dataloader_4d_set_num_samples(flexmi_dataloader_4d_t d, int n) { return flexmi_dataloader_set_num_samples(d, n); }
void flexmi_dataloader_4d_destroy(flexmi_dataloader_4d_t d) { flexmi_dataloader_destroy(d); }
int flexmi_dataloader_2d_next_batch(flexmi_dataloader_2d_t d, flexmi_model_t m) { return flexmi_dataloader_next_batch(d, m); }
int flexmi_dataloader_2d_reset(flexmi_dataloader_2d_t d) { return flexmi_dataloader_reset(d); }
int flexmi_dataloader_2d_get_num_samples(flexmi_dataloader_2d_t d) { return flexmi_dataloader_get_num_samples(d); }
int flexmi_dataloader_2d_set_num_samples(flexmi_dataloader_2d_t d, int n) { return flexmi_dataloader_set_num_samples(d, n); }
void flexmi_dataloader_2d_destroy(flexmi_dataloader_2d_t d) { flexmi_dataloader_destroy(d); }
int flexmi_single_dataloader_reset(flexmi_single_dataloader_t d) { return flexmi_dataloader_reset(d); }
int flexmi_single_dataloader_get_num_samples(flexmi_single_dataloader_t d) { return flexmi_dataloader_get_num_samples(d); }
int flexmi_single_dataloader_set_num_samples(flexmi_single_dataloader_t d, int n) {
  return flexmi_dataloader_set_num_samples(d, n);
}
void flexmi_single_dataloader_destroy(flexmi_single_dataloader_t d) { flexmi_dataloader_destroy(d); }

}  // extern "C"


// mjcf_embed.cpp -- libmpcr_mjcf.so: the MJCF -> mpcr_model_t compiler behind
// the C ABI (mpcr_model_load on an .xml path; MjModel.from_xml_path,
// SBP/mjx_planner.py:100-103).  The compiler itself is the package's
// manipulator_mujoco_amd/mjcf.py (includes, default classes, mesh inertia,
// convex hulls through scipy's Qhull, pair filtering, mj_setConst-style
// constants); this library runs it in an embedded CPython so that a host
// without Python code of its own (C, C++, Go over cgo, ...) can load a scene
// from its MJCF.  libmpcr.so dlopens it only when it is handed an .xml path,
// so the rollout engine itself never links Python.
//
// Host side only (g++, no HIP).  Thread-safe: one compile at a time.
#include <Python.h>
#include <dlfcn.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>

namespace {

std::mutex g_mu;

void set_err(char* err, int errlen, const std::string& msg) {
  if (err && errlen > 0) std::snprintf(err, (size_t)errlen, "%s", msg.c_str());
}

// the package root: <root>/manipulator_mujoco_amd/libmpcr_mjcf.so
std::string package_root() {
  Dl_info info;
  if (!dladdr(reinterpret_cast<void*>(&package_root), &info) || !info.dli_fname) return ".";
  std::string p(info.dli_fname);
  for (int k = 0; k < 2; k++) {
    size_t s = p.find_last_of('/');
    p = s == std::string::npos ? std::string(".") : p.substr(0, s);
  }
  return p;
}

std::string py_error() {
  PyObject *type = nullptr, *value = nullptr, *tb = nullptr;
  PyErr_Fetch(&type, &value, &tb);
  std::string msg = "python error";
  if (value) {
    PyObject* s = PyObject_Str(value);
    if (s) {
      const char* c = PyUnicode_AsUTF8(s);
      if (c) msg = c;
      Py_DECREF(s);
    }
  }
  Py_XDECREF(type);
  Py_XDECREF(value);
  Py_XDECREF(tb);
  return msg;
}

}  // namespace

extern "C" {

// Compile the MJCF at `path` (timestep <= 0: the file's own <option
// timestep>) into a serialised mpcr_model_t.  *blob is malloc'd (free with
// mpcr_mjcf_free); returns 0, or -1 with a message in err.
int mpcr_mjcf_compile(const char* path, double timestep, void** blob, size_t* nbytes, char* err, int errlen) {
  if (!path || !blob || !nbytes) {
    set_err(err, errlen, "null argument");
    return -1;
  }
  std::lock_guard<std::mutex> lock(g_mu);
  if (!Py_IsInitialized()) {
    // a host without an interpreter: start one and hand the GIL back, so
    // every call below takes it through PyGILState_Ensure like a Python host.
    // libpython came in as a dependency of a RTLD_LOCAL dlopen: promote it to
    // global scope first, or extension modules (numpy, _ctypes) cannot
    // resolve the interpreter's symbols
    Dl_info pi;
    if (dladdr(reinterpret_cast<void*>(&Py_InitializeEx), &pi) && pi.dli_fname)
      dlopen(pi.dli_fname, RTLD_NOW | RTLD_GLOBAL | RTLD_NOLOAD);
    Py_InitializeEx(0);
    PyEval_SaveThread();
  }
  PyGILState_STATE gs = PyGILState_Ensure();
  int rc = -1;
  PyObject *sys_path = nullptr, *root = nullptr, *mod = nullptr, *res = nullptr;
  do {
    sys_path = PySys_GetObject("path");  // borrowed
    root = PyUnicode_FromString(package_root().c_str());
    if (!sys_path || !root) { set_err(err, errlen, "sys.path unavailable"); break; }
    if (PySequence_Contains(sys_path, root) == 0 && PyList_Insert(sys_path, 0, root) != 0) {
      set_err(err, errlen, py_error());
      break;
    }
    mod = PyImport_ImportModule("manipulator_mujoco_amd.mjcf");
    if (!mod) { set_err(err, errlen, "import manipulator_mujoco_amd.mjcf: " + py_error()); break; }
    res = PyObject_CallMethod(mod, "compile_blob", "sd", path, timestep);
    if (!res) { set_err(err, errlen, py_error()); break; }
    char* data = nullptr;
    Py_ssize_t len = 0;
    if (PyBytes_AsStringAndSize(res, &data, &len) != 0) { set_err(err, errlen, py_error()); break; }
    void* out = std::malloc((size_t)len);
    if (!out) { set_err(err, errlen, "out of memory"); break; }
    std::memcpy(out, data, (size_t)len);
    *blob = out;
    *nbytes = (size_t)len;
    rc = 0;
  } while (false);
  Py_XDECREF(res);
  Py_XDECREF(mod);
  Py_XDECREF(root);
  PyGILState_Release(gs);
  return rc;
}

void mpcr_mjcf_free(void* blob) { std::free(blob); }

}  // extern "C"

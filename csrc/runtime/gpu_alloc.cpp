// Gang GPU placement core for the local MI355X node (part of kubedl_amd._native).
//
// best_fit(free_mask, n, group_masks) -> mask of the n GPUs to grant, or -1.
//
// Policy (see kubedl_amd/gang/allocator.py): a request that fits inside one
// host-locality group (the two 4-GPU halves of an 8 x MI355X platform, one per
// CPU socket) goes to the group with the FEWEST free GPUs that still fits
// (best fit keeps whole halves free for later 4-GPU gangs); otherwise the n
// lowest free GPUs.  xGMI connects every GPU pair directly, so inside a group
// the choice does not change collective bandwidth.  Bitmasks hold up to 64 GPUs.
#define PY_SSIZE_T_CLEAN
#include <Python.h>

#include <stdint.h>

#include <vector>

namespace {

int popcount64(uint64_t v) { return __builtin_popcountll(v); }

uint64_t lowest_n(uint64_t m, int n) {
  uint64_t out = 0;
  for (int i = 0; i < 64 && n > 0; ++i) {
    if (m & (1ull << i)) {
      out |= 1ull << i;
      --n;
    }
  }
  return n == 0 ? out : 0;
}

PyObject* py_best_fit(PyObject*, PyObject* args) {
  unsigned long long free_mask;
  int n;
  PyObject* groups;
  if (!PyArg_ParseTuple(args, "KiO", &free_mask, &n, &groups)) return nullptr;
  if (n < 0) {
    PyErr_SetString(PyExc_ValueError, "n must be >= 0");
    return nullptr;
  }
  if (n == 0) return PyLong_FromLong(0);
  PyObject* fast = PySequence_Fast(groups, "group_masks must be a sequence of int");
  if (!fast) return nullptr;
  std::vector<uint64_t> gm;
  for (Py_ssize_t i = 0; i < PySequence_Fast_GET_SIZE(fast); ++i) {
    unsigned long long v = PyLong_AsUnsignedLongLong(PySequence_Fast_GET_ITEM(fast, i));
    if (PyErr_Occurred()) {
      Py_DECREF(fast);
      return nullptr;
    }
    gm.push_back(v);
  }
  Py_DECREF(fast);
  int best = -1, best_avail = 65;
  for (size_t g = 0; g < gm.size(); ++g) {
    const int avail = popcount64(free_mask & gm[g]);
    if (avail >= n && avail < best_avail) {
      best = static_cast<int>(g);
      best_avail = avail;
    }
  }
  uint64_t chosen = 0;
  if (best >= 0) chosen = lowest_n(free_mask & gm[best], n);
  else if (popcount64(free_mask) >= n) chosen = lowest_n(free_mask, n);
  if (chosen == 0) return PyLong_FromLong(-1);
  return PyLong_FromUnsignedLongLong(chosen);
}

PyMethodDef alloc_methods[] = {
    {"best_fit", py_best_fit, METH_VARARGS,
     "best_fit(free_mask, n, group_masks) -> granted GPU bitmask, or -1 if it cannot fit"},
    {nullptr, nullptr, 0, nullptr}};

}  // namespace

extern "C" PyObject* kdl_native_alloc_module_init(PyObject* m) {
  if (PyModule_AddFunctions(m, alloc_methods) != 0) return nullptr;
  return m;
}

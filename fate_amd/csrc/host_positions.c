/* Host-side index work of the vector ops (no device code; loaded through ctypes.PyDLL).
 *
 * 1. Marshalling of the reference's position lists for CiphertextVector::iupdate /
 * iupdate_with_masks (fixedpoint_paillier/src/lib.rs:724-747; paillier.rs:261-283 takes them
 * as Vec<Vec<usize>>, which pyo3 extracts element by element).  SecureBoost hands them over
 * as Python lists of lists (HistogramIndexer.get_positions, arch/histogram/
 * _histogram_local.py:68-82): ~4M Python ints for a 1M-sample, 4-feature histogram.  These
 * two calls walk them once each under the GIL (loaded through ctypes.PyDLL) and write plain
 * int64 arrays that go to the device as they are; the Python-level flattening they replace
 * took ~0.8 s for that shape, 50x the device fold.
 *
 * Both return -1 with a Python exception set on a malformed argument (not a sequence, an
 * element that is not an integer, a value outside int64); ranges are the caller's check. */
#include <Python.h>
#include <stdint.h>

/* Both passes walk a private tuple snapshot of the outer sequence (PySequence_Tuple holds
 * strong references).  An inner list of plain ints -- the usual case -- is read in place: no
 * Python code can run while it is read.  Any other inner sequence, or one holding other
 * integer types (whose __index__ may run Python code), is read from its own tuple snapshot. */

/* lens[i] = len(outer[i]) for i < len(outer) (lens has room for cap entries: a list that grew
 * since the caller sized it is an error); returns the sum */
int64_t fphe_py_positions_lens(PyObject* outer, int64_t* lens, int64_t cap) {
  PyObject* o = PySequence_Tuple(outer);
  if (!o) return -1;
  const Py_ssize_t n = PyTuple_GET_SIZE(o);
  if ((int64_t)n != cap) {
    Py_DECREF(o);
    PyErr_SetString(PyExc_RuntimeError, "positions changed while being read");
    return -1;
  }
  int64_t total = 0;
  for (Py_ssize_t i = 0; i < n; ++i) {
    PyObject* in = PyTuple_GET_ITEM(o, i);
    const Py_ssize_t k = PyList_CheckExact(in) ? PyList_GET_SIZE(in) : PySequence_Size(in);
    if (k < 0) {
      Py_DECREF(o);
      return -1;
    }
    lens[i] = (int64_t)k;
    total += (int64_t)k;
  }
  Py_DECREF(o);
  return total;
}

/* pos[j] = the j-th listed position, sample-major as the reference walks them; `total` is
 * what fphe_py_positions_lens returned (a list that changed in between is an error) */
int64_t fphe_py_positions_fill(PyObject* outer, int64_t* pos, int64_t total) {
  PyObject* o = PySequence_Tuple(outer);
  if (!o) return -1;
  const Py_ssize_t n = PyTuple_GET_SIZE(o);
  int64_t j = 0;
  for (Py_ssize_t i = 0; i < n; ++i) {
    PyObject* li = PyTuple_GET_ITEM(o, i);
    if (PyList_CheckExact(li)) {  /* in place while every item is a plain int */
      const Py_ssize_t k = PyList_GET_SIZE(li);
      Py_ssize_t t = 0;
      if (j + (int64_t)k <= total) {
        for (; t < k; ++t) {
          PyObject* v = PyList_GET_ITEM(li, t);
          if (!PyLong_CheckExact(v)) break;
          const long long x = PyLong_AsLongLong(v);
          if (x == -1 && PyErr_Occurred()) {
            Py_DECREF(o);
            return -1;
          }
          pos[j + t] = (int64_t)x;
        }
        if (t == k) {
          j += k;
          continue;
        }
      }
    }
    PyObject* in = PySequence_Tuple(li);
    if (!in) {
      Py_DECREF(o);
      return -1;
    }
    const Py_ssize_t k = PyTuple_GET_SIZE(in);
    if (j + (int64_t)k > total) {
      Py_DECREF(in);
      Py_DECREF(o);
      PyErr_SetString(PyExc_RuntimeError, "positions changed while being read");
      return -1;
    }
    for (Py_ssize_t t = 0; t < k; ++t) {
      const long long x = PyLong_AsLongLong(PyTuple_GET_ITEM(in, t)); /* __index__ for numpy ints */
      if (x == -1 && PyErr_Occurred()) {
        Py_DECREF(in);
        Py_DECREF(o);
        return -1;
      }
      pos[j++] = (int64_t)x;
    }
    Py_DECREF(in);
  }
  Py_DECREF(o);
  if (j != total) {
    PyErr_SetString(PyExc_RuntimeError, "positions changed while being read");
    return -1;
  }
  return total;
}

/* 2. CiphertextVector::i_shuffle's cycle walk (fixedpoint_paillier/src/lib.rs:473-490) on
 * positions instead of ciphertexts: perm[k] = the original element that ends at k, so the
 * device does one gather.  The walk is the reference's, swap for swap, so any index list --
 * not only a permutation -- gives the reference's result.  Returns 0, or 1 at the first
 * access the reference would panic on, with bad[0] = the length indexed and bad[1] = the
 * index ("index out of bounds: the len is .. but the index is .."): indexes[i] past the list
 * (nix < n), or visited[next] past the data.  Indexes are non-negative (usize). */
int fphe_cycle_walk(const int64_t* ix, int64_t nix, int64_t n, int64_t* perm, uint8_t* visited, int64_t* bad) {
  for (int64_t k = 0; k < n; ++k) {
    perm[k] = k;
    visited[k] = 0;
  }
  for (int64_t i = 0; i < n; ++i) {
    if (visited[i]) continue;
    if (i >= nix) {
      bad[0] = nix;
      bad[1] = i;
      return 1;
    }
    if (ix[i] == i) continue;
    int64_t current = i, next = ix[current];
    for (;;) {
      if (next >= n) {
        bad[0] = n;
        bad[1] = next;
        return 1;
      }
      if (visited[next] || next == i) break;
      const int64_t t = perm[current];
      perm[current] = perm[next];
      perm[next] = t;
      visited[current] = 1;
      current = next;
      if (current >= nix) {
        bad[0] = nix;
        bad[1] = current;
        return 1;
      }
      next = ix[current];
    }
    visited[current] = 1;
  }
  return 0;
}

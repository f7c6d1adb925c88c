// ffddp_pybind.cpp — pybind11 module over the C ABI (include/ffddp.h), the
// boundary SURVEY.md §7 step 4 / §8(b) names beside the C entry points.
//
// `_ffddp_native.Solver` is crocoddyl.SolverBoxFDDP(problem) for a batch
// (crocoddyl_classical.py:442-445): `solve` takes the same numpy arrays as
// ffddp_solve_batch (crocoddyl_classical.py:365-388 batched) and returns the
// read-backs as new arrays.  The GIL is released for the duration of the
// device solve, so several Python threads can drive handles on different
// GPUs.  Host code only: it links libffddp.so (the HIP kernels) and adds no
// device code of its own; errors raise RuntimeError with ffddp_last_error.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>

#include <cstring>
#include <stdexcept>
#include <string>

#include "ffddp.h"

namespace py = pybind11;

namespace {

using f64 = py::array_t<double, py::array::c_style | py::array::forcecast>;
using u8 = py::array_t<uint8_t, py::array::c_style | py::array::forcecast>;

template <class T> T struct_from(const py::buffer& b, const char* what) {
  const py::buffer_info bi = b.request();
  const size_t n = (size_t)bi.size * (size_t)bi.itemsize;
  if (n != sizeof(T))
    throw std::invalid_argument(std::string(what) + ": expected " + std::to_string(sizeof(T)) + " bytes, got " +
                                std::to_string(n));
  T t;
  std::memcpy(&t, bi.ptr, sizeof(T));
  return t;
}

void check_shape(const py::array& a, std::initializer_list<py::ssize_t> shape, const char* name) {
  if ((size_t)a.ndim() != shape.size()) throw std::invalid_argument(std::string(name) + ": wrong number of dimensions");
  size_t i = 0;
  for (py::ssize_t s : shape) {
    if (a.shape(i) != s) throw std::invalid_argument(std::string(name) + ": wrong shape");
    ++i;
  }
}

class Solver {
 public:
  // robot, cfg: the bytes of an ffddp_robot / ffddp_ocp_config (e.g.
  // bytes(ffddp._abi.make_robot()), bytes(OcpConfig.to_struct()))
  Solver(const py::buffer& robot, const py::buffer& cfg, int device, int max_batch) {
    rb_ = struct_from<ffddp_robot>(robot, "robot");
    cfg_ = struct_from<ffddp_ocp_config>(cfg, "cfg");
    const int rc = ffddp_create(&rb_, &cfg_, device, max_batch, &h_);
    if (rc != 0) throw std::runtime_error("ffddp_create failed (" + std::to_string(rc) + ")");
    N_ = cfg_.horizon;
    nx_ = cfg_.variant == FFDDP_FORCE_FEEDBACK ? 21 : 14;
    max_batch_ = max_batch;
  }
  ~Solver() { close(); }
  Solver(const Solver&) = delete;
  Solver& operator=(const Solver&) = delete;

  void close() {
    if (h_) {
      ffddp_destroy(h_);
      h_ = nullptr;
    }
  }

  py::dict solve(const f64& x0, const f64& node_ref, const f64& inst_ref, const u8& surface, const f64& xs_init,
                 const f64& us_init, int maxiter, bool is_feasible) {
    if (!h_) throw std::runtime_error("solver is closed");
    const py::ssize_t B = x0.ndim() == 2 ? x0.shape(0) : -1;
    if (B < 0 || B > max_batch_) throw std::invalid_argument("x0: expected [B][nx] with B <= max_batch");
    const py::ssize_t N = N_, nx = nx_;
    check_shape(x0, {B, nx}, "x0");
    check_shape(node_ref, {B, N + 1, 6}, "node_ref");
    check_shape(inst_ref, {B, 21}, "inst_ref");
    check_shape(surface, {B}, "surface");
    check_shape(xs_init, {B, N + 1, nx}, "xs_init");
    check_shape(us_init, {B, N, FFDDP_NU}, "us_init");
    f64 xs({B, N + 1, nx}), us({B, N, (py::ssize_t)FFDDP_NU}), K({B, N, (py::ssize_t)FFDDP_NU, nx}), cost({B}),
        fn({B, (py::ssize_t)2});
    py::array_t<int32_t> iters({B}), stats({B, (py::ssize_t)FFDDP_NSTATS});
    py::array_t<uint8_t> ok({B});
    int rc;
    {
      py::gil_scoped_release nogil;
      rc = ffddp_solve_batch(h_, (int)B, x0.data(), node_ref.data(), inst_ref.data(), surface.data(), xs_init.data(),
                             us_init.data(), maxiter, is_feasible ? 1 : 0, xs.mutable_data(), us.mutable_data(),
                             K.mutable_data(), cost.mutable_data(), iters.mutable_data(), ok.mutable_data(),
                             fn.mutable_data(), stats.mutable_data());
    }
    if (rc != 0) {
      const char* msg = ffddp_last_error(h_);
      throw std::runtime_error("ffddp_solve_batch failed (" + std::to_string(rc) + "): " + (msg ? msg : ""));
    }
    py::dict out;
    out["xs"] = xs;
    out["us"] = us;
    out["K"] = K;
    out["cost"] = cost;
    out["iter"] = iters;
    out["ok"] = ok;
    out["fn_pred"] = fn;
    out["stats"] = stats;
    return out;
  }

  int N() const { return N_; }
  int nx() const { return nx_; }
  int max_batch() const { return max_batch_; }

 private:
  ffddp_handle* h_ = nullptr;
  ffddp_robot rb_{};
  ffddp_ocp_config cfg_{};
  int N_ = 0, nx_ = 0, max_batch_ = 0;
};

}  // namespace

PYBIND11_MODULE(_ffddp_native, m) {
  m.doc() = "pybind11 binding of the batched (Box)FDDP C ABI (include/ffddp.h)";
  m.attr("NSTATS") = FFDDP_NSTATS;
  m.attr("ROBOT_BYTES") = sizeof(ffddp_robot);
  m.attr("CFG_BYTES") = sizeof(ffddp_ocp_config);
  py::class_<Solver>(m, "Solver")
      .def(py::init<const py::buffer&, const py::buffer&, int, int>(), py::arg("robot"), py::arg("cfg"),
           py::arg("device") = 0, py::arg("max_batch") = 1)
      .def("solve", &Solver::solve, py::arg("x0"), py::arg("node_ref"), py::arg("inst_ref"), py::arg("surface"),
           py::arg("xs_init"), py::arg("us_init"), py::arg("maxiter") = 10, py::arg("is_feasible") = false,
           "Batched SolverBoxFDDP.solve on host arrays (ffddp_solve_batch); the GIL is released during the solve.")
      .def("close", &Solver::close)
      .def_property_readonly("N", &Solver::N)
      .def_property_readonly("nx", &Solver::nx)
      .def_property_readonly("max_batch", &Solver::max_batch);
}

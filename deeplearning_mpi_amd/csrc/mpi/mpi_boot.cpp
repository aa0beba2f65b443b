// MPI bootstrap module `deeplearning_mpi_amd._mpi` (pybind11 + libmpi, no torch dependency).
//
// Under `mpirun`, ranks are discovered from MPI itself (MPI_Comm_rank / a shared-memory split for
// the node-local rank), the RCCL unique id is distributed with MPI_Bcast, and host-side
// collectives (the CPU "hello world" all-reduce, plain barriers) go straight through MPI.  The
// reference has no MPI at all (it is torchrun-only); this is the launcher
// substrate BASELINE.json asks for.
#include <mpi.h>
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>

#include <stdexcept>
#include <string>

namespace py = pybind11;

static void mpi_check(int rc, const char* what) {
  if (rc != MPI_SUCCESS) {
    char msg[MPI_MAX_ERROR_STRING];
    int len = 0;
    MPI_Error_string(rc, msg, &len);
    throw std::runtime_error(std::string("MPI ") + what + " failed: " + std::string(msg, len));
  }
}

static bool is_initialized() {
  int f = 0;
  MPI_Initialized(&f);
  return f != 0;
}

static py::tuple init() {
  if (!is_initialized()) {
    int provided = 0;
    mpi_check(MPI_Init_thread(nullptr, nullptr, MPI_THREAD_MULTIPLE, &provided), "MPI_Init_thread");
  }
  int rank = 0, size = 1;
  MPI_Comm_rank(MPI_COMM_WORLD, &rank);
  MPI_Comm_size(MPI_COMM_WORLD, &size);
  return py::make_tuple(rank, size);
}

static py::tuple local_rank() {
  MPI_Comm node;
  mpi_check(MPI_Comm_split_type(MPI_COMM_WORLD, MPI_COMM_TYPE_SHARED, 0, MPI_INFO_NULL, &node), "split_type");
  int lr = 0, ls = 1;
  MPI_Comm_rank(node, &lr);
  MPI_Comm_size(node, &ls);
  MPI_Comm_free(&node);
  return py::make_tuple(lr, ls);
}

static py::bytes bcast_bytes(const std::string& data, int root) {
  int rank = 0;
  MPI_Comm_rank(MPI_COMM_WORLD, &rank);
  long long n = (long long)data.size();
  mpi_check(MPI_Bcast(&n, 1, MPI_LONG_LONG, root, MPI_COMM_WORLD), "MPI_Bcast(size)");
  std::string buf = rank == root ? data : std::string((size_t)n, '\0');
  if (n > 0) mpi_check(MPI_Bcast(&buf[0], (int)n, MPI_BYTE, root, MPI_COMM_WORLD), "MPI_Bcast");
  return py::bytes(buf);
}

template <typename T>
static void allreduce_arr(py::array_t<T, py::array::c_style> a, const std::string& op, MPI_Datatype dt) {
  MPI_Op o = MPI_SUM;
  if (op == "max") o = MPI_MAX;
  else if (op == "min") o = MPI_MIN;
  else if (op == "prod") o = MPI_PROD;
  else if (op != "sum") throw std::runtime_error("allreduce: unknown op " + op);
  auto buf = a.request(true);
  mpi_check(MPI_Allreduce(MPI_IN_PLACE, buf.ptr, (int)buf.size, dt, o, MPI_COMM_WORLD), "MPI_Allreduce");
}

static void send_arr(py::array_t<float, py::array::c_style> a, int dst, int tag) {
  auto b = a.request();
  mpi_check(MPI_Send(b.ptr, (int)b.size, MPI_FLOAT, dst, tag, MPI_COMM_WORLD), "MPI_Send");
}
static void recv_arr(py::array_t<float, py::array::c_style> a, int src, int tag) {
  auto b = a.request(true);
  mpi_check(MPI_Recv(b.ptr, (int)b.size, MPI_FLOAT, src, tag, MPI_COMM_WORLD, MPI_STATUS_IGNORE), "MPI_Recv");
}

static std::string processor_name() {
  char name[MPI_MAX_PROCESSOR_NAME];
  int len = 0;
  MPI_Get_processor_name(name, &len);
  return std::string(name, len);
}

PYBIND11_MODULE(_mpi, m) {
  m.doc() = "MPI bootstrap for deeplearning_mpi_amd";
  m.def("initialized", &is_initialized);
  m.def("init", &init);
  m.def("local_rank", &local_rank);
  m.def("bcast_bytes", &bcast_bytes, py::arg("data"), py::arg("root") = 0);
  m.def("allreduce_f64", [](py::array_t<double, py::array::c_style> a, const std::string& op) {
    allreduce_arr<double>(a, op, MPI_DOUBLE);
  }, py::arg("a"), py::arg("op") = "sum");
  m.def("allreduce_f32", [](py::array_t<float, py::array::c_style> a, const std::string& op) {
    allreduce_arr<float>(a, op, MPI_FLOAT);
  }, py::arg("a"), py::arg("op") = "sum");
  m.def("send_f32", &send_arr, py::arg("a"), py::arg("dst"), py::arg("tag") = 0);
  m.def("recv_f32", &recv_arr, py::arg("a"), py::arg("src"), py::arg("tag") = 0);
  m.def("barrier", []() { mpi_check(MPI_Barrier(MPI_COMM_WORLD), "MPI_Barrier"); });
  m.def("finalize", []() {
    int f = 0;
    MPI_Finalized(&f);
    if (is_initialized() && !f) MPI_Finalize();
  });
  m.def("processor_name", &processor_name);
}

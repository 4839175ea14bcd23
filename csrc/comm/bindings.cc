// pybind11 module mivod._mvcomm: mivod's RCCL data plane.  Tensors cross the
// boundary as raw device pointers (tensor.data_ptr()) and HIP streams as
// handles (torch.cuda.Stream.cuda_stream); no torch headers are needed.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "comm.h"
#include "mesh.h"

namespace py = pybind11;
using namespace mvcomm;

PYBIND11_MODULE(_mvcomm, m) {
  m.doc() = "mivod GPU data plane: RCCL communicator, collectives on the comm stream, watchdog";
  m.def("unique_id", [] { return py::bytes(unique_id()); });
  m.def("rccl_version", &rccl_version);
  m.def("header_version", [] { return (int)NCCL_VERSION_CODE; });
  m.def("version_note", &version_note);

  // ncclDataType_t / ncclRedOp_t codes (rccl.h)
  m.attr("INT8") = (int)ncclInt8;
  m.attr("UINT8") = (int)ncclUint8;
  m.attr("INT32") = (int)ncclInt32;
  m.attr("UINT32") = (int)ncclUint32;
  m.attr("INT64") = (int)ncclInt64;
  m.attr("UINT64") = (int)ncclUint64;
  m.attr("FLOAT16") = (int)ncclFloat16;
  m.attr("FLOAT32") = (int)ncclFloat32;
  m.attr("FLOAT64") = (int)ncclFloat64;
  m.attr("BFLOAT16") = (int)ncclBfloat16;
  m.attr("SUM") = (int)ncclSum;
  m.attr("PROD") = (int)ncclProd;
  m.attr("MAX") = (int)ncclMax;
  m.attr("MIN") = (int)ncclMin;
  m.attr("AVG") = (int)ncclAvg;

  py::class_<CommStats>(m, "CommStats")
      .def_readonly("calls", &CommStats::calls)
      .def_readonly("bytes", &CommStats::bytes)
      .def_readonly("completed", &CommStats::completed);

  py::class_<Comm>(m, "Comm")
      .def(py::init([](py::bytes uid, int rank, int size, int device, double timeout_s,
                       bool exit_on_abort, int min_ctas, int max_ctas) {
             std::string u = uid;
             py::gil_scoped_release nogil;
             return std::make_unique<Comm>(u, rank, size, device, timeout_s, exit_on_abort,
                                           min_ctas, max_ctas);
           }),
           py::arg("uid"), py::arg("rank"), py::arg("size"), py::arg("device"),
           py::arg("timeout_s") = 0.0, py::arg("exit_on_abort") = false,
           py::arg("min_ctas") = 0, py::arg("max_ctas") = 0)
      .def_property_readonly("min_ctas", &Comm::min_ctas)
      .def_property_readonly("max_ctas", &Comm::max_ctas)
      .def_property_readonly("rank", &Comm::rank)
      .def_property_readonly("size", &Comm::size)
      .def_property_readonly("device", &Comm::device)
      .def("count", &Comm::count)
      .def("allreduce",
           [](Comm& c, uintptr_t in, uintptr_t out, size_t n, int dt, int op, uintptr_t s) {
             c.allreduce((const void*)in, (void*)out, n, dt, op, s);
           },
           py::call_guard<py::gil_scoped_release>())
      .def("allreduce_premul",
           [](Comm& c, uintptr_t in, uintptr_t out, size_t n, int dt, double scale,
              uintptr_t s) { c.allreduce_premul((const void*)in, (void*)out, n, dt, scale, s); },
           py::call_guard<py::gil_scoped_release>())
      .def("reduce_scatter",
           [](Comm& c, uintptr_t in, uintptr_t out, size_t n, int dt, int op, uintptr_t s) {
             c.reduce_scatter((const void*)in, (void*)out, n, dt, op, s);
           },
           py::call_guard<py::gil_scoped_release>())
      .def("allgather",
           [](Comm& c, uintptr_t in, uintptr_t out, size_t n, int dt, uintptr_t s) {
             c.allgather((const void*)in, (void*)out, n, dt, s);
           },
           py::call_guard<py::gil_scoped_release>())
      .def("broadcast",
           [](Comm& c, uintptr_t in, uintptr_t out, size_t n, int dt, int root, uintptr_t s) {
             c.broadcast((const void*)in, (void*)out, n, dt, root, s);
           },
           py::call_guard<py::gil_scoped_release>())
      .def("sendrecv",
           [](Comm& c, uintptr_t sb, size_t sn, uintptr_t rb, size_t rn, int dt, int peer,
              uintptr_t s) { c.sendrecv((const void*)sb, sn, (void*)rb, rn, dt, peer, s); },
           py::call_guard<py::gil_scoped_release>())
      .def("alltoallv",
           [](Comm& c, uintptr_t sb, std::vector<size_t> sc, std::vector<size_t> sd, uintptr_t rb,
              std::vector<size_t> rc, std::vector<size_t> rd, int dt, uintptr_t s) {
             c.alltoallv((const void*)sb, sc, sd, (void*)rb, rc, rd, dt, s);
           },
           py::call_guard<py::gil_scoped_release>())
      .def("split",
           [](Comm& c, int color, int key) {
             py::gil_scoped_release nogil;
             return c.split(color, key);
           })
      .def("check", &Comm::check)
      .def("error", &Comm::error)
      .def("abort", &Comm::abort, py::call_guard<py::gil_scoped_release>())
      .def("destroy", &Comm::destroy, py::call_guard<py::gil_scoped_release>())
      .def("stats", &Comm::stats)
      .def("outstanding", &Comm::outstanding);

  // xGMI mesh allreduce (one-shot / two-shot) over HIP-IPC-mapped peer buffers
  py::class_<Mesh>(m, "Mesh")
      .def(py::init<int, int, int, size_t, double, bool>(), py::arg("rank"), py::arg("size"),
           py::arg("device"), py::arg("capacity_bytes"), py::arg("timeout_s") = 30.0,
           py::arg("exit_on_timeout") = true)
      .def("handles", [](const Mesh& me) { return py::bytes(me.handles()); })
      .def("open",
           [](Mesh& me, std::vector<py::bytes> hs) {
             std::vector<std::string> v;
             for (auto& h : hs) v.push_back(std::string(h));
             py::gil_scoped_release nogil;
             me.open(v);
           })
      .def("stage_ptr", &Mesh::stage_ptr)
      .def("allreduce",
           [](Mesh& me, uintptr_t in, uintptr_t out, size_t n, int dt, float scale, uintptr_t s,
              int algo) { me.allreduce((const void*)in, (void*)out, n, dt, scale, s, algo); },
           py::arg("inp"), py::arg("out"), py::arg("count"), py::arg("dtype"), py::arg("scale"),
           py::arg("stream"), py::arg("algo") = 0, py::call_guard<py::gil_scoped_release>())
      .def("status", &Mesh::status)
      .def("failed", &Mesh::failed)
      .def("close", &Mesh::close, py::call_guard<py::gil_scoped_release>())
      .def_property("oneshot_max_bytes", &Mesh::oneshot_max_bytes, &Mesh::set_oneshot_max_bytes)
      .def_property_readonly("capacity", &Mesh::capacity)
      .def_property_readonly("timeout_s", &Mesh::timeout_s)
      .def_property_readonly("rank", &Mesh::rank)
      .def_property_readonly("size", &Mesh::size)
      .def_property_readonly("calls", &Mesh::calls)
      .def_property_readonly("bytes", &Mesh::bytes)
      .def_property_readonly("copies_saved", &Mesh::copies_saved)
      .def_property_readonly("two_shot_calls", &Mesh::two_shot_calls);
}

// pybind11 module mivod._mvcore: the native engine core (no GPU dependency).
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "controller.h"
#include "loop.h"
#include "ring.h"
#include "store.h"
#include "timeline.h"

namespace py = pybind11;
using namespace mvcore;

namespace {

// request tuple: (name, kind, dtype, shape, root, op, device, nbytes[, prescale, postscale])
Request to_request(const py::handle& h) {
  auto t = py::reinterpret_borrow<py::tuple>(h);
  if (t.size() != 8 && t.size() != 10)
    throw std::invalid_argument("mivod request must be an 8- or 10-tuple");
  Request r;
  r.name = t[0].cast<std::string>();
  r.kind = (uint8_t)t[1].cast<int>();
  r.dtype = t[2].cast<std::string>();
  for (auto d : t[3]) r.shape.push_back(d.cast<int64_t>());
  r.root = t[4].cast<int32_t>();
  r.op = t[5].cast<int32_t>();
  r.device = t[6].cast<int32_t>();
  r.nbytes = t[7].cast<int64_t>();
  if (t.size() == 10) {
    r.prescale = t[8].cast<double>();
    r.postscale = t[9].cast<double>();
  }
  return r;
}

py::list to_py(const std::vector<Response>& rs) {
  py::list out;
  for (const auto& r : rs) {
    py::list names;
    for (const auto& n : r.names) names.append(n);
    out.append(py::make_tuple((int)r.kind, names, r.error));
  }
  return out;
}

}  // namespace

PYBIND11_MODULE(_mvcore, m) {
  m.doc() = "mivod native engine core: TCP coordinator, stall inspector, timeline";

  py::class_<Timeline, std::shared_ptr<Timeline>>(m, "Timeline")
      .def(py::init<const std::string&, bool>(), py::arg("path"), py::arg("mark_cycles") = false)
      .def("start", &Timeline::start, py::arg("name"), py::arg("phase"), py::arg("args") = "",
           py::call_guard<py::gil_scoped_release>())
      .def("activity", &Timeline::activity, py::call_guard<py::gil_scoped_release>())
      .def("end", &Timeline::end, py::call_guard<py::gil_scoped_release>())
      .def("instant", &Timeline::instant, py::call_guard<py::gil_scoped_release>())
      .def("complete", &Timeline::complete, py::call_guard<py::gil_scoped_release>())
      .def("now_us", &Timeline::now_us)
      .def("mark_cycle", &Timeline::mark_cycle, py::call_guard<py::gil_scoped_release>())
      .def("close", &Timeline::close, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("events_written", &Timeline::events_written);

  // CPU data plane: ring collectives over TCP on raw host pointers (tensor.data_ptr())
  // rendezvous key-value store (launcher-hosted server, one client per rank)
  py::class_<KVServer>(m, "KVServer")
      .def(py::init<const std::string&, int>(), py::arg("host") = "0.0.0.0", py::arg("port") = 0)
      .def_property_readonly("port", &KVServer::port)
      .def_property_readonly("requests", &KVServer::requests)
      .def("close", &KVServer::close, py::call_guard<py::gil_scoped_release>());
  py::class_<KVClient>(m, "KVClient")
      .def(py::init([](const std::string& host, int port, double timeout_s) {
             py::gil_scoped_release nogil;
             return std::make_unique<KVClient>(host, port, timeout_s);
           }),
           py::arg("host"), py::arg("port"), py::arg("timeout_s") = 300.0)
      .def("set",
           [](KVClient& c, const std::string& k, py::bytes v) {
             std::string s = v;
             py::gil_scoped_release nogil;
             c.set(k, s);
           })
      .def("get",
           [](KVClient& c, const std::string& k) {
             std::string v;
             {
               py::gil_scoped_release nogil;
               v = c.get(k);
             }
             return py::bytes(v);
           })
      .def("add", &KVClient::add, py::call_guard<py::gil_scoped_release>())
      .def("check", &KVClient::check, py::call_guard<py::gil_scoped_release>())
      .def("wait", &KVClient::wait, py::call_guard<py::gil_scoped_release>())
      .def("delete_key", &KVClient::remove, py::call_guard<py::gil_scoped_release>())
      .def("num_keys", &KVClient::num_keys, py::call_guard<py::gil_scoped_release>())
      .def("compare_set",
           [](KVClient& c, const std::string& k, py::bytes e, py::bytes d) {
             std::string es = e, ds = d, v;
             {
               py::gil_scoped_release nogil;
               v = c.compare_set(k, es, ds);
             }
             return py::bytes(v);
           })
      .def("set_timeout", &KVClient::set_timeout)
      .def_property_readonly("timeout", &KVClient::timeout)
      .def("close", &KVClient::close, py::call_guard<py::gil_scoped_release>());

  py::class_<Ring>(m, "Ring")
      .def(py::init<int, int, double>(), py::arg("rank"), py::arg("size"),
           py::arg("timeout_s") = 300.0)
      .def("listen", &Ring::listen, py::call_guard<py::gil_scoped_release>())
      .def("connect", &Ring::connect, py::call_guard<py::gil_scoped_release>())
      .def("allreduce",
           [](Ring& r, uintptr_t ptr, int64_t count, int dtype, bool average) {
             r.allreduce((void*)ptr, count, dtype, average);
           },
           py::arg("ptr"), py::arg("count"), py::arg("dtype"), py::arg("average") = false,
           py::call_guard<py::gil_scoped_release>())
      .def("allgatherv",
           [](Ring& r, uintptr_t in, uintptr_t out, std::vector<int64_t> bytes) {
             r.allgatherv((const void*)in, (void*)out, bytes);
           },
           py::call_guard<py::gil_scoped_release>())
      .def("broadcast",
           [](Ring& r, uintptr_t ptr, int64_t bytes, int root) {
             r.broadcast((void*)ptr, bytes, root);
           },
           py::call_guard<py::gil_scoped_release>())
      .def("barrier", &Ring::barrier, py::call_guard<py::gil_scoped_release>())
      .def("set_timeout", &Ring::set_timeout)
      .def("close", &Ring::close, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("rank", &Ring::rank)
      .def_property_readonly("size", &Ring::size)
      .def_property_readonly("bytes_sent", &Ring::bytes_sent);
  m.def("ring_reduce_sum",
        [](uintptr_t dst, uintptr_t src, int64_t n, int dtype) {
          ring_reduce_sum((void*)dst, (const void*)src, n, dtype);
        },
        "dst += src (host reducer of the CPU ring; fp16 via F16C, bf16 via fp32 RNE)");

  py::class_<ControllerConfig>(m, "ControllerConfig")
      .def(py::init<>())
      .def_readwrite("rank", &ControllerConfig::rank)
      .def_readwrite("size", &ControllerConfig::size)
      .def_readwrite("host", &ControllerConfig::host)
      .def_readwrite("port", &ControllerConfig::port)
      .def_readwrite("fusion_threshold", &ControllerConfig::fusion_threshold)
      .def_readwrite("stall_check_s", &ControllerConfig::stall_check_s)
      .def_readwrite("stall_shutdown_s", &ControllerConfig::stall_shutdown_s)
      .def_readwrite("stall_check", &ControllerConfig::stall_check)
      .def_readwrite("connect_timeout_s", &ControllerConfig::connect_timeout_s)
      .def_readwrite("cache_capacity", &ControllerConfig::cache_capacity);

  py::class_<Controller, std::shared_ptr<Controller>>(m, "Controller")
      .def(py::init<const ControllerConfig&>())
      .def("listen", &Controller::listen, py::call_guard<py::gil_scoped_release>())
      .def("connect", &Controller::connect, py::call_guard<py::gil_scoped_release>())
      .def("set_timeline", &Controller::set_timeline)
      .def("negotiate",
           [](Controller& c, py::list reqs, bool shutdown, int64_t position) {
             std::vector<Request> rs;
             rs.reserve(reqs.size());
             for (auto h : reqs) rs.push_back(to_request(h));
             bool all = false;
             int64_t exec_at = position;
             std::vector<Response> out;
             {
               py::gil_scoped_release nogil;
               out = c.negotiate(rs, shutdown, &all, position, &exec_at);
             }
             return py::make_tuple(to_py(out), all, exec_at);
           },
           py::arg("requests"), py::arg("shutdown") = false, py::arg("position") = 0)
      .def("coordinate_for_test",
           [](Controller& c, py::list per_rank) {
             std::vector<std::vector<Request>> pr;
             for (auto lst : per_rank) {
               std::vector<Request> rs;
               for (auto h : lst) rs.push_back(to_request(h));
               pr.push_back(rs);
             }
             return to_py(c.coordinate_for_test(pr));
           })
      .def("last_stalls",
           [](const Controller& c) {
             py::list out;
             for (const auto& s : c.last_stalls())
               out.append(py::make_tuple(s.name, s.missing_ranks, s.age_s));
             return out;
           })
      .def_property_readonly("cycles", &Controller::cycles)
      .def_property_readonly("cache_hits", &Controller::cache_hits)
      .def_property_readonly("bitvector_cycles", &Controller::bitvector_cycles)
      .def_property_readonly("cache_size", &Controller::cache_size)
      .def("close", &Controller::close, py::call_guard<py::gil_scoped_release>());

  // background negotiation loop (native thread; Python executes the responses)
  py::class_<EngineLoop>(m, "EngineLoop")
      .def(py::init<std::shared_ptr<Controller>, int, double>(), py::arg("controller"),
           py::arg("size"), py::arg("cycle_s"))
      .def("submit",
           [](EngineLoop& l, py::list reqs) {
             std::vector<Request> rs;
             rs.reserve(reqs.size());
             for (auto h : reqs) rs.push_back(to_request(h));
             py::gil_scoped_release nogil;
             l.submit(std::move(rs));
           })
      .def("set_position", &EngineLoop::set_position)
      .def("request_shutdown", &EngineLoop::request_shutdown,
           py::call_guard<py::gil_scoped_release>())
      .def("wait",
           [](EngineLoop& l, double timeout_s) -> py::object {
             CycleResult r;
             bool ok;
             {
               py::gil_scoped_release nogil;
               ok = l.wait(timeout_s, &r);
             }
             if (!ok) return py::none();
             return py::make_tuple(to_py(r.responses), r.all_shutdown, r.exec_at, r.error);
           },
           py::arg("timeout_s") = -1.0)
      .def("join", &EngineLoop::join, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("finished", &EngineLoop::finished)
      .def_property_readonly("cycles", &EngineLoop::cycles)
      .def_property_readonly("requests", &EngineLoop::requests);
}

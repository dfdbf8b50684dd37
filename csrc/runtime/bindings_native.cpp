// pybind11 module ps_amd._native: TCP parameter server / client, id map, batch loader.
// Every blocking call releases the GIL so Python worker threads (prefetch, UI) keep running.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "loader.h"
#include "ps_server.h"

namespace py = pybind11;
using namespace psnative;

namespace {

using F32 = py::array_t<float, py::array::c_style | py::array::forcecast>;
using I64 = py::array_t<int64_t, py::array::c_style | py::array::forcecast>;

py::array_t<float> to_array(const Matrix& m) {
  py::array_t<float> a({static_cast<py::ssize_t>(m.rows), static_cast<py::ssize_t>(m.cols)});
  std::memcpy(a.mutable_data(), m.data.data(), m.data.size() * sizeof(float));
  return a;
}

void put_mat(Writer& w, const F32& a) {
  uint32_t rows = 1, cols = 1;
  if (a.ndim() == 1) {
    rows = static_cast<uint32_t>(a.shape(0));
  } else if (a.ndim() == 2) {
    rows = static_cast<uint32_t>(a.shape(0));
    cols = static_cast<uint32_t>(a.shape(1));
  } else if (a.ndim() == 0) {
    rows = cols = 1;
  } else {
    rows = static_cast<uint32_t>(a.shape(0));
    cols = static_cast<uint32_t>(a.size() / a.shape(0));
  }
  w.mat(rows, cols, a.data());
}

void check(uint16_t st, const std::vector<uint8_t>& resp, const char* what) {
  if (st == ST_OK || st == ST_NOT_FOUND) return;
  std::string msg;
  if (!resp.empty()) {
    try {
      Reader r(resp.data(), resp.size());
      msg = r.str();
    } catch (...) {
    }
  }
  if (st == ST_TIMEOUT) throw std::runtime_error(std::string(what) + ": timed out (dead worker?)");
  throw std::runtime_error(std::string(what) + " failed (" + std::to_string(st) + "): " + msg);
}

class Client {
 public:
  Client(const std::string& host, int port, double timeout) : c_(host, port, timeout) {}

  py::object get(const std::string& key) {
    Writer w;
    w.str(key);
    std::vector<uint8_t> resp;
    uint16_t st;
    {
      py::gil_scoped_release r;
      st = c_.call(OP_GET, w, &resp);
    }
    check(st, resp, "get");
    if (st == ST_NOT_FOUND) return py::none();
    Reader rd(resp.data(), resp.size());
    return to_array(rd.mat());
  }

  py::list get_list(const std::vector<std::string>& keys) {
    Writer w;
    w.u32(static_cast<uint32_t>(keys.size()));
    for (auto& k : keys) w.str(k);
    std::vector<uint8_t> resp;
    uint16_t st;
    {
      py::gil_scoped_release r;
      st = c_.call(OP_GET_LIST, w, &resp);
    }
    check(st, resp, "get_list");
    Reader rd(resp.data(), resp.size());
    const uint32_t n = rd.u32();
    py::list out;
    for (uint32_t i = 0; i < n; ++i) {
      if (rd.u8()) out.append(to_array(rd.mat()));
      else out.append(py::none());
    }
    return out;
  }

  py::tuple upsert(const std::string& key, const F32& a, bool replace) {
    Writer w;
    w.u8(replace ? 1 : 0);
    w.str(key);
    put_mat(w, a);
    std::vector<uint8_t> resp;
    uint16_t st;
    {
      py::gil_scoped_release r;
      st = c_.call(OP_UPSERT, w, &resp);
    }
    check(st, resp, "upsert");
    Reader rd(resp.data(), resp.size());
    const bool existed = rd.u8() != 0;
    return py::make_tuple(existed, to_array(rd.mat()));
  }

  py::list upsert_list(const std::vector<std::string>& keys, const std::vector<F32>& arrs, bool replace) {
    if (keys.size() != arrs.size()) throw std::runtime_error("keys/arrays length mismatch");
    Writer w;
    w.u8(replace ? 1 : 0);
    w.u32(static_cast<uint32_t>(keys.size()));
    for (size_t i = 0; i < keys.size(); ++i) {
      w.str(keys[i]);
      put_mat(w, arrs[i]);
    }
    std::vector<uint8_t> resp;
    uint16_t st;
    {
      py::gil_scoped_release r;
      st = c_.call(OP_UPSERT_LIST, w, &resp);
    }
    check(st, resp, "upsert_list");
    Reader rd(resp.data(), resp.size());
    const uint32_t n = rd.u32();
    py::list out;
    for (uint32_t i = 0; i < n; ++i) {
      const bool existed = rd.u8() != 0;
      out.append(py::make_tuple(existed, to_array(rd.mat())));
    }
    return out;
  }

  void push(const std::vector<std::string>& keys, const std::vector<F32>& grads, const std::string& spec,
            int async_flag) {
    if (keys.size() != grads.size()) throw std::runtime_error("keys/grads length mismatch");
    Writer w;
    w.u8(static_cast<uint8_t>(async_flag));
    w.str(spec);
    w.u32(static_cast<uint32_t>(keys.size()));
    for (size_t i = 0; i < keys.size(); ++i) {
      w.str(keys[i]);
      put_mat(w, grads[i]);
    }
    std::vector<uint8_t> resp;
    uint16_t st;
    {
      py::gil_scoped_release r;
      st = c_.call(OP_PUSH, w, &resp);
    }
    check(st, resp, "push");
  }

  uint64_t barrier(uint32_t worker) {
    Writer w;
    w.u32(worker);
    std::vector<uint8_t> resp;
    uint16_t st;
    {
      py::gil_scoped_release r;
      st = c_.call(OP_BARRIER, w, &resp);
    }
    check(st, resp, "barrier");
    Reader rd(resp.data(), resp.size());
    return rd.u64();
  }

  uint64_t clock(uint32_t worker, uint64_t c) {
    Writer w;
    w.u32(worker);
    w.u64(c);
    std::vector<uint8_t> resp;
    uint16_t st;
    {
      py::gil_scoped_release r;
      st = c_.call(OP_CLOCK, w, &resp);
    }
    check(st, resp, "clock");
    Reader rd(resp.data(), resp.size());
    return rd.u64();
  }

  py::array_t<float> row_pull(const std::string& table, uint32_t dim, const I64& keys, float lo, float hi,
                              uint64_t seed) {
    Writer w;
    w.str(table);
    w.u32(dim);
    w.f32(lo);
    w.f32(hi);
    w.u64(seed);
    w.u32(static_cast<uint32_t>(keys.size()));
    w.raw(keys.data(), static_cast<size_t>(keys.size()) * 8);
    std::vector<uint8_t> resp;
    uint16_t st;
    {
      py::gil_scoped_release r;
      st = c_.call(OP_ROW_PULL, w, &resp);
    }
    check(st, resp, "row_pull");
    Reader rd(resp.data(), resp.size());
    const uint32_t n = rd.u32();
    py::array_t<float> out({static_cast<py::ssize_t>(n), static_cast<py::ssize_t>(dim)});
    std::vector<float> tmp;
    rd.vec(&tmp, static_cast<size_t>(n) * dim);
    std::memcpy(out.mutable_data(), tmp.data(), tmp.size() * sizeof(float));
    return out;
  }

  void row_push(const std::string& table, uint32_t dim, const I64& keys, const F32& grads, const std::string& spec,
                int async_flag) {
    if (static_cast<size_t>(grads.size()) != static_cast<size_t>(keys.size()) * dim)
      throw std::runtime_error("row_push: grads must be [n, dim]");
    Writer w;
    w.u8(static_cast<uint8_t>(async_flag));
    w.str(spec);
    w.str(table);
    w.u32(dim);
    w.u32(static_cast<uint32_t>(keys.size()));
    w.raw(keys.data(), static_cast<size_t>(keys.size()) * 8);
    w.f32s(grads.data(), static_cast<size_t>(grads.size()));
    std::vector<uint8_t> resp;
    uint16_t st;
    {
      py::gil_scoped_release r;
      st = c_.call(OP_ROW_PUSH, w, &resp);
    }
    check(st, resp, "row_push");
  }

  void simple(Op op, const std::string& s) {
    Writer w;
    w.str(s);
    std::vector<uint8_t> resp;
    uint16_t st;
    {
      py::gil_scoped_release r;
      st = c_.call(op, w, &resp);
    }
    check(st, resp, "request");
  }

  std::string stats() {
    Writer w;
    std::vector<uint8_t> resp;
    uint16_t st = c_.call(OP_STATS, w, &resp);
    check(st, resp, "stats");
    Reader rd(resp.data(), resp.size());
    return rd.str();
  }

  void heartbeat(uint32_t worker) {
    Writer w;
    w.u32(worker);
    std::vector<uint8_t> resp;
    check(c_.call(OP_HEARTBEAT, w, &resp), resp, "heartbeat");
  }

  void shutdown() {
    Writer w;
    std::vector<uint8_t> resp;
    c_.call(OP_SHUTDOWN, w, &resp);
  }

  uint64_t bytes_sent() const { return c_.bytes_sent(); }
  uint64_t bytes_recv() const { return c_.bytes_recv(); }

 private:
  PSClient c_;
};

py::object batch_to_dict(Batch& b, int dims, int fields) {
  py::dict d;
  const py::ssize_t n = b.n;
  if (!b.x.empty()) {
    py::array_t<float> x({n, static_cast<py::ssize_t>(dims)});
    std::memcpy(x.mutable_data(), b.x.data(), b.x.size() * 4);
    d["X"] = x;
  }
  if (!b.i.empty()) {
    py::array_t<int64_t> i({n, static_cast<py::ssize_t>(fields)});
    std::memcpy(i.mutable_data(), b.i.data(), b.i.size() * 8);
    d["I"] = i;
  }
  if (!b.v.empty()) {
    py::array_t<float> v({n, static_cast<py::ssize_t>(fields)});
    std::memcpy(v.mutable_data(), b.v.data(), b.v.size() * 4);
    d["V"] = v;
  }
  py::array_t<float> y(n);
  std::memcpy(y.mutable_data(), b.y.data(), b.y.size() * 4);
  d["Y"] = y;
  return d;
}

}  // namespace

PYBIND11_MODULE(_native, m) {
  m.doc() = "ps_amd native CPU runtime: TCP parameter server/client, id map, threaded batch loader";

  py::class_<PSServer>(m, "PSServer")
      .def(py::init<int, int, const std::string&, int, double>(), py::arg("port") = 0, py::arg("workers") = 1,
           py::arg("mode") = "bsp", py::arg("staleness") = 0, py::arg("barrier_timeout_s") = 600.0)
      .def("start", &PSServer::start)
      .def("stop", &PSServer::stop, py::call_guard<py::gil_scoped_release>())
      .def("wait", &PSServer::wait, py::call_guard<py::gil_scoped_release>())
      .def("set_bind_any", &PSServer::set_bind_any)
      .def_property_readonly("port", &PSServer::port)
      .def_property_readonly("generation", &PSServer::generation)
      .def_property_readonly("updates", &PSServer::updates);

  py::class_<Client>(m, "PSClient")
      .def(py::init<const std::string&, int, double>(), py::arg("host"), py::arg("port"),
           py::arg("timeout_s") = 30.0)
      .def("get", &Client::get)
      .def("get_list", &Client::get_list)
      .def("upsert", &Client::upsert, py::arg("key"), py::arg("value"), py::arg("replace") = false)
      .def("upsert_list", &Client::upsert_list, py::arg("keys"), py::arg("values"), py::arg("replace") = false)
      .def("push", &Client::push, py::arg("keys"), py::arg("grads"), py::arg("spec"), py::arg("async_flag") = 0)
      .def("barrier", &Client::barrier, py::arg("worker") = 0)
      .def("clock", &Client::clock)
      .def("row_pull", &Client::row_pull, py::arg("table"), py::arg("dim"), py::arg("keys"), py::arg("lo"),
           py::arg("hi"), py::arg("seed"))
      .def("row_push", &Client::row_push, py::arg("table"), py::arg("dim"), py::arg("keys"), py::arg("grads"),
           py::arg("spec"), py::arg("async_flag") = 0)
      .def("register_updater", [](Client& c, const std::string& s) { c.simple(OP_REGISTER, s); })
      .def("save", [](Client& c, const std::string& p) { c.simple(OP_SAVE, p); })
      .def("load", [](Client& c, const std::string& p) { c.simple(OP_LOAD, p); })
      .def("stats", &Client::stats)
      .def("heartbeat", &Client::heartbeat)
      .def("shutdown", &Client::shutdown)
      .def_property_readonly("bytes_sent", &Client::bytes_sent)
      .def_property_readonly("bytes_recv", &Client::bytes_recv);

  py::class_<IdMap>(m, "IdMap")
      .def(py::init<int64_t>())
      .def("lookup",
           [](IdMap& self, const I64& ids, bool insert) {
             py::array_t<int64_t> out(ids.size());
             {
               py::gil_scoped_release r;
               self.lookup(ids.data(), ids.size(), insert, out.mutable_data());
             }
             return out;
           },
           py::arg("ids"), py::arg("insert") = true)
      .def("size", &IdMap::size)
      .def("items", &IdMap::items)
      .def("restore", [](IdMap& self, const I64& ids, const I64& slots) {
        if (ids.size() != slots.size()) throw std::runtime_error("ids/slots length mismatch");
        self.restore(ids.data(), slots.data(), ids.size());
      });

  py::class_<BatchReader>(m, "BatchReader")
      .def(py::init<const std::string&, const std::string&, int, int, int, int, int, int, int, bool>(),
           py::arg("path"), py::arg("format"), py::arg("batch"), py::arg("dims") = 0, py::arg("fields") = 0,
           py::arg("offset") = 0, py::arg("step") = 1, py::arg("threads") = 2, py::arg("depth") = 4,
           py::arg("drop_last") = false)
      .def("next",
           [](BatchReader& self, double timeout) -> py::object {
             Batch b;
             bool ok;
             {
               py::gil_scoped_release r;
               ok = self.next(&b, timeout);
             }
             if (!ok) return py::none();
             return batch_to_dict(b, self.dims(), self.fields());
           },
           py::arg("timeout_s") = 3.0)
      .def("has_next", &BatchReader::has_next, py::call_guard<py::gil_scoped_release>())
      .def("reset", &BatchReader::reset, py::call_guard<py::gil_scoped_release>());
}

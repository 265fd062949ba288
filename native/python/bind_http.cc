// pybind11 surface of the HTTP stack (native/core/http.cc, http2.cc, net.cc) for the unit
// tests: a TLS test server with a few behaviours (echo, slow, large, chunked) and the
// native client, so HTTP/1.1 and HTTP/2 (ALPN h2) paths — multiplexing, flow control,
// graceful drain, reconnects, stream resets — are exercised without the services.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <atomic>
#include <chrono>
#include <memory>
#include <thread>

#include "core/http.h"
#include "core/net.h"

namespace py = pybind11;

namespace bgc_py {

namespace {

class TestServer {
 public:
  TestServer(const std::string& cert_pem, const std::string& key_pem, bool http2, int idle_timeout_ms,
             std::vector<std::string> inline_paths) {
    bgc::http::ServerOptions so;
    so.addr = "127.0.0.1";
    so.port = 0;
    so.name = "http-test";
    so.http2 = http2;
    so.h2_inline_paths = std::move(inline_paths);
    if (idle_timeout_ms > 0) so.idle_timeout_ms = idle_timeout_ms;
    if (!cert_pem.empty()) so.tls = bgc::net::TlsContext::server_from_pem(cert_pem, key_pem);
    srv_ = std::make_unique<bgc::http::Server>(so);
    // POST /echo: the body back, with the protocol that carried it
    srv_->handle("POST", "/echo", [this](bgc::http::Request& r, bgc::http::ResponseWriter& w) {
      ++served_;
      bgc::http::Headers h;
      h.set("X-Protocol", w.protocol());
      h.set("X-Echo-Query", r.query);
      w.send(200, r.body, "application/octet-stream", &h);
    });
    // GET /slow?ms=N: answers after N ms (a request in flight during stop())
    srv_->handle("GET", "/slow", [this](bgc::http::Request& r, bgc::http::ResponseWriter& w) {
      std::this_thread::sleep_for(std::chrono::milliseconds(std::stoi(r.query_param("ms", "100"))));
      ++served_;
      w.send(200, "done");
    });
    // GET /big?n=N: N bytes (more than the peer's flow-control window)
    srv_->handle("GET", "/big", [this](bgc::http::Request& r, bgc::http::ResponseWriter& w) {
      ++served_;
      std::string body(std::stoul(r.query_param("n", "1")), 'x');
      for (size_t i = 0; i < body.size(); i += 4096) body[i] = static_cast<char>('a' + (i / 4096) % 26);
      w.send(200, body, "application/octet-stream");
    });
    // GET /chunks?n=N: N newline-terminated lines as a streamed (chunked / DATA) response
    srv_->handle("GET", "/chunks", [this](bgc::http::Request& r, bgc::http::ResponseWriter& w) {
      ++served_;
      int n = std::stoi(r.query_param("n", "3"));
      w.start_chunked(200, "application/json");
      for (int i = 0; i < n && !w.peer_closed(); ++i) w.write_chunk("{\"i\":" + std::to_string(i) + "}\n");
      w.end_chunked();
    });
    srv_->start();
  }
  uint16_t port() const { return srv_->port(); }
  uint64_t served() const { return served_.load(); }
  uint64_t inline_served() const { return srv_->h2_inline_served(); }
  void stop(int grace_ms) { srv_->stop(std::chrono::milliseconds(grace_ms)); }

 private:
  std::unique_ptr<bgc::http::Server> srv_;
  std::atomic<uint64_t> served_{0};
};

}  // namespace

void register_http(py::module_& m) {
  py::class_<TestServer>(m, "HttpTestServer")
      .def(py::init<const std::string&, const std::string&, bool, int, std::vector<std::string>>(), py::arg("cert_pem"),
           py::arg("key_pem"), py::arg("http2") = true, py::arg("idle_timeout_ms") = 0,
           py::arg("inline_paths") = std::vector<std::string>{})
      .def_property_readonly("port", &TestServer::port)
      .def_property_readonly("inline_served", &TestServer::inline_served)
      .def_property_readonly("served", &TestServer::served)
      .def("stop", &TestServer::stop, py::arg("grace_ms") = 10000, py::call_guard<py::gil_scoped_release>());

  py::class_<bgc::http::Client>(m, "HttpClient")
      .def(py::init([](const std::string& base_url, const std::string& ca_pem, bool http2, size_t h2_connections,
                       int timeout_ms, bool h2_caller_reads) {
             bgc::http::ClientOptions o;
             o.base_url = base_url;
             o.http2 = http2;
             o.h2_connections = h2_connections;
             o.timeout_ms = timeout_ms;
             o.h2_caller_reads = h2_caller_reads;
             if (base_url.rfind("https", 0) == 0) o.tls = bgc::net::TlsContext::client(ca_pem, false);
             return std::make_unique<bgc::http::Client>(o);
           }),
           py::arg("base_url"), py::arg("ca_pem") = "", py::arg("http2") = true, py::arg("h2_connections") = 1,
           py::arg("timeout_ms") = 10000, py::arg("h2_caller_reads") = false)
      // (status, body bytes, {lowercased header: value}); raises RuntimeError (HttpError) on
      // transport failures and timeouts
      .def("request",
           [](bgc::http::Client& c, const std::string& method, const std::string& path, const py::bytes& body,
              int timeout_ms) {
             std::string b = body;
             bgc::http::Response r;
             {
               py::gil_scoped_release nogil;
               r = c.request(method, path, b, nullptr, timeout_ms);
             }
             py::dict h;
             for (auto& [k, v] : r.headers.items()) {
               std::string lk = k;
               for (auto& ch : lk) ch = static_cast<char>(std::tolower(static_cast<unsigned char>(ch)));
               h[py::str(lk)] = v;
             }
             return py::make_tuple(r.status, py::bytes(r.body), h);
           },
           py::arg("method"), py::arg("path"), py::arg("body") = py::bytes(), py::arg("timeout_ms") = -1)
      .def("close_idle", &bgc::http::Client::close_idle);
}

}  // namespace bgc_py

#include "bench/churn.h"

#include <algorithm>
#include <array>
#include <future>
#include <random>
#include <thread>

#include "core/log.h"
#include "core/metrics.h"
#include "core/net.h"
#include "core/trace.h"
#include "kube/runtime.h"

namespace bgc::bench {

using json::Value;
namespace types = kube::types;

ChurnDriver::ChurnDriver(ChurnOptions o) : opts_(std::move(o)) {
  kube::KubeConfig kc;
  kc.server = opts_.server;
  kc.token = opts_.admin_token;
  kc.ca_pem = opts_.ca_pem;
  kc.timeout_ms = 60000;
  kc.http2 = opts_.http2;
  admin_ = std::make_unique<kube::KubeClient>(kc);
  http::ClientOptions ho;
  ho.base_url = opts_.server;
  ho.timeout_ms = 60000;
  ho.max_idle = static_cast<size_t>(opts_.concurrency) * 2;
  ho.http2 = opts_.http2;
  if (opts_.server.rfind("https", 0) == 0) ho.tls = net::TlsContext::client(opts_.ca_pem, false, "", "");
  http_ = std::make_unique<http::Client>(ho);
  pool_ = std::make_unique<ThreadPool>(static_cast<size_t>(std::max(1, opts_.concurrency)), "drv-create");
  delete_pool_ = std::make_unique<ThreadPool>(static_cast<size_t>(std::max(1, opts_.concurrency / 2)), "drv-delete");
}

json::Value ChurnDriver::step_with_delete(const std::vector<std::string>& names,
                                          const std::vector<std::string>& previous, double timeout_s) {
  std::vector<std::future<bool>> dels;
  for (const auto& n : previous) {
    dels.push_back(delete_pool_->submit([this, n] {
      try {
        admin_->remove(types::UserBootstrap, "", n);
        return true;
      } catch (const kube::ApiError& e) {
        return e.code() == 404;
      } catch (const std::exception&) {
        return false;
      }
    }));
  }
  Value out = step(names, timeout_s);
  int failures = 0;
  for (auto& f : dels) failures += f.get() ? 0 : 1;
  {
    std::lock_guard<std::mutex> lk(mu_);
    for (const auto& n : previous) early_.erase(n);
  }
  out["delete_failures"] = failures;
  return out;
}

ChurnDriver::~ChurnDriver() { stop(); }

void ChurnDriver::mark(const std::string& name, int which, int64_t t) {
  if (name.compare(0, opts_.name_prefix.size(), opts_.name_prefix) != 0) return;
  std::lock_guard<std::mutex> lk(mu_);
  auto it = tracks_.find(name);
  if (it == tracks_.end()) {
    auto& e = early_[name];
    if (!e[static_cast<size_t>(which)]) e[static_cast<size_t>(which)] = t;
    return;
  }
  Track& tr = it->second;
  int64_t* slot = which == 0 ? &tr.t_ns : which == 1 ? &tr.t_rq : &tr.t_rb;
  if (*slot) return;
  *slot = t;
  if (trace::armed()) trace::mark_at(name, which == 0 ? "drv.ns_seen" : which == 1 ? "drv.rq_seen" : "drv.rb_seen", t);
  if (tr.delete_when_ready && ready_locked(tr)) issue_delete(name);
  // approve-after-create waits on Namespaces alone; otherwise only Ready matters
  if (ready_locked(tr) || (which == 0 && !opts_.approve_url.empty())) cv_.notify_all();
}

void ChurnDriver::issue_delete(const std::string& name) {
  delete_pool_->submit([this, name] {
    try {
      admin_->remove(types::UserBootstrap, "", name);
    } catch (const kube::ApiError& e) {
      if (e.code() != 404) delete_failures_.fetch_add(1);
    } catch (const std::exception&) {
      delete_failures_.fetch_add(1);
    }
  });
}

void ChurnDriver::start() {
  struct W {
    const kube::ResourceType* rt;
    int which;
  };
  for (W w : {W{&types::Namespace, 0}, W{&types::ResourceQuota, 1}, W{&types::RoleBinding, 2}}) {
    watchers_.emplace_back([this, w] {
      const bool filter = opts_.server_filter && !opts_.name_prefix.empty();
      kube::Watcher watcher(*admin_, *w.rt, "", "", filter ? "kube-lite.test/name-prefix=" + opts_.name_prefix : "");
      if (!opts_.name_prefix.empty()) {
        // one driver per rank: skip other ranks' tenants without parsing their events
        // (each child's name, and its owner reference, carry the tenant name)
        std::string needle = "\"name\":\"" + opts_.name_prefix;
        watcher.set_line_filter([needle](std::string_view l) { return l.find(needle) != std::string_view::npos; });
      }
      std::string key = opts_.gpu_quota_key;
      watcher.run(stop_, [&](const kube::WatchEvent& ev) {
        auto handle = [&](const Value& o) {
          std::string name = kube::meta_name(o);
          if (w.which == 1 && !o.get("spec").get("hard").contains(key)) return;
          mark(name, w.which, metrics::now_ns());
        };
        if (ev.type == kube::WatchEvent::Type::Restarted) {
          for (const auto& o : ev.objects) handle(*o);
        } else if (ev.type != kube::WatchEvent::Type::Deleted) {
          handle(*ev.object);
        }
      });
    });
  }
}

json::Value ChurnDriver::step(const std::vector<std::string>& names, double timeout_s) {
  int64_t t0 = metrics::now_ns();
  {
    std::lock_guard<std::mutex> lk(mu_);
    for (const auto& n : names) {
      Track t;
      t.t_start = t0;
      auto e = early_.find(n);
      if (e != early_.end()) {
        t.t_ns = e->second[0];
        t.t_rq = e->second[1];
        t.t_rb = e->second[2];
        early_.erase(e);
      }
      tracks_[n] = t;
    }
  }
  std::vector<std::future<void>> futs;
  futs.reserve(names.size());
  for (const auto& n : names) {
    futs.push_back(pool_->submit([this, n] {
      int64_t ts = metrics::now_ns();
      Value body = Value::object({{"apiVersion", "bacchus.io/v1"}, {"kind", "UserBootstrap"},
                                  {"metadata", Value::object({{"name", n}})}, {"spec", Value::object()}});
      http::Headers h;
      h.set("Authorization", "Bearer " + opts_.admin_token);
      h.set("Impersonate-User", opts_.user_prefix + n);
      h.set("Impersonate-Group", opts_.group);
      h.set("Content-Type", "application/json");
      std::string err;
      try {
        http::Response r = http_->request("POST", types::UserBootstrap.collection_path(), body.dump(), &h);
        if (r.status != 201 && r.status != 200) err = std::to_string(r.status) + " " + r.body;
      } catch (const std::exception& e) {
        err = e.what();
      }
      std::lock_guard<std::mutex> lk(mu_);
      Track& t = tracks_[n];
      t.t_start = ts;
      t.t_created = metrics::now_ns();
      if (!err.empty()) {
        t.failed = true;
        t.error = err;
      }
      cv_.notify_all();
    }));
  }
  for (auto& f : futs) f.get();
  auto deadline = std::chrono::steady_clock::now() +
                  std::chrono::duration_cast<std::chrono::steady_clock::duration>(std::chrono::duration<double>(timeout_s));
  if (!opts_.approve_url.empty()) approve_batch(names, deadline);
  Value out = Value::object();
  std::unique_lock<std::mutex> lk(mu_);
  auto all_done = [&] {
    for (const auto& n : names) {
      const Track& t = tracks_[n];
      if (!t.failed && !ready_locked(t)) return false;
    }
    return true;
  };
  cv_.wait_until(lk, deadline, all_done);
  int64_t t_end = metrics::now_ns();
  Value lat = Value::array(), clat = Value::array(), errs = Value::array();
  Value ns_lat = Value::array(), rq_lat = Value::array(), rb_lat = Value::array();
  Value ap_lat = Value::array(), ap_ready = Value::array();
  int ready = 0, failed = 0, timeouts = 0;
  int64_t last_ready = t0;
  for (const auto& n : names) {
    const Track& t = tracks_[n];
    if (t.failed) {
      ++failed;
      if (errs.size() < 5) errs.push_back(n + ": " + t.error);
    } else if (ready_locked(t)) {
      ++ready;
      int64_t tr = std::max({t.t_ns, t.t_rq, t.t_rb});
      last_ready = std::max(last_ready, tr);
      lat.push_back(static_cast<double>(tr - t.t_start) * 1e-9);
      clat.push_back(static_cast<double>(t.t_created - t.t_start) * 1e-9);
      ns_lat.push_back(static_cast<double>(t.t_ns - t.t_start) * 1e-9);
      rq_lat.push_back(static_cast<double>(t.t_rq - t.t_start) * 1e-9);
      rb_lat.push_back(static_cast<double>(t.t_rb - t.t_start) * 1e-9);
      if (t.t_approved) {
        ap_lat.push_back(static_cast<double>(t.t_approved - t.t_start) * 1e-9);
        ap_ready.push_back(static_cast<double>(tr - t.t_approved) * 1e-9);
      }
    } else {
      ++timeouts;
    }
    tracks_.erase(n);
  }
  out["ready"] = ready;
  out["failed"] = failed;
  out["timeouts"] = timeouts;
  out["elapsed_s"] = static_cast<double>((ready == static_cast<int>(names.size()) ? last_ready : t_end) - t0) * 1e-9;
  out["ready_latency_s"] = lat;
  out["create_latency_s"] = clat;
  out["ns_latency_s"] = ns_lat;  // stage breakdown: Namespace, quota'd ResourceQuota, RoleBinding seen
  out["rq_latency_s"] = rq_lat;
  out["rb_latency_s"] = rb_lat;
  out["errors"] = errs;
  if (!opts_.approve_url.empty()) {
    out["approve_latency_s"] = ap_lat;
    out["approve_to_ready_latency_s"] = ap_ready;
  }
  return out;
}

json::Value ChurnDriver::open_loop(const std::vector<std::string>& names, double duration_s, double timeout_s,
                                   uint64_t seed) {
  const size_t n = names.size();
  std::vector<int64_t> offset(n);
  {
    std::mt19937_64 rng(seed);
    std::uniform_real_distribution<double> u(0.0, duration_s * 1e9);
    for (auto& o : offset) o = static_cast<int64_t>(u(rng));
    std::sort(offset.begin(), offset.end());
  }
  delete_failures_.store(0);
  const int64_t t0 = metrics::now_ns() + 2000000;  // 2 ms to register the tracks first
  {
    std::lock_guard<std::mutex> lk(mu_);
    for (size_t i = 0; i < n; ++i) {
      Track t;
      t.t_start = t0 + offset[i];
      t.delete_when_ready = opts_.approve_url.empty();
      tracks_[names[i]] = t;
    }
  }
  std::vector<int64_t> lag(n);
  std::vector<std::future<void>> futs;
  futs.reserve(n);
  const auto base = std::chrono::steady_clock::now() + std::chrono::nanoseconds(t0 - metrics::now_ns());
  for (size_t i = 0; i < n; ++i) {
    std::this_thread::sleep_until(base + std::chrono::nanoseconds(offset[i]));
    lag[i] = metrics::now_ns() - (t0 + offset[i]);
    const std::string& name = names[i];
    if (trace::armed()) trace::mark_at(name, "drv.sched", t0 + offset[i]);
    futs.push_back(pool_->submit([this, name] {
      if (trace::armed()) trace::mark(name, "drv.sent");
      Value body = Value::object({{"apiVersion", "bacchus.io/v1"}, {"kind", "UserBootstrap"},
                                  {"metadata", Value::object({{"name", name}})}, {"spec", Value::object()}});
      http::Headers h;
      h.set("Authorization", "Bearer " + opts_.admin_token);
      h.set("Impersonate-User", opts_.user_prefix + name);
      h.set("Impersonate-Group", opts_.group);
      h.set("Content-Type", "application/json");
      std::string err;
      try {
        http::Response r = http_->request("POST", types::UserBootstrap.collection_path(), body.dump(), &h);
        if (r.status != 201 && r.status != 200) err = std::to_string(r.status) + " " + r.body;
      } catch (const std::exception& e) {
        err = e.what();
      }
      std::lock_guard<std::mutex> lk(mu_);
      Track& t = tracks_[name];
      t.t_created = metrics::now_ns();
      if (trace::armed()) trace::mark_at(name, "drv.created", t.t_created);
      if (!err.empty()) {
        t.failed = true;
        t.error = err;
      }
      cv_.notify_all();
    }));
  }
  for (auto& f : futs) f.get();
  const auto deadline = std::chrono::steady_clock::now() +
                        std::chrono::duration_cast<std::chrono::steady_clock::duration>(std::chrono::duration<double>(timeout_s));
  Value out = Value::object();
  std::unique_lock<std::mutex> lk(mu_);
  cv_.wait_until(lk, deadline, [&] {
    for (const auto& nm : names) {
      const Track& t = tracks_[nm];
      if (!t.failed && !ready_locked(t)) return false;
    }
    return true;
  });
  Value lat = Value::array(), clat = Value::array(), errs = Value::array();
  Value ns_lat = Value::array(), rq_lat = Value::array(), rb_lat = Value::array();
  int ready = 0, failed = 0, timeouts = 0;
  int64_t last_ready = t0;
  for (const auto& nm : names) {
    const Track& t = tracks_[nm];
    if (t.failed) {
      ++failed;
      if (errs.size() < 5) errs.push_back(nm + ": " + t.error);
    } else if (ready_locked(t)) {
      ++ready;
      const int64_t tr = std::max({t.t_ns, t.t_rq, t.t_rb});
      last_ready = std::max(last_ready, tr);
      lat.push_back(static_cast<double>(tr - t.t_start) * 1e-9);
      clat.push_back(static_cast<double>(t.t_created - t.t_start) * 1e-9);
      ns_lat.push_back(static_cast<double>(t.t_ns - t.t_start) * 1e-9);
      rq_lat.push_back(static_cast<double>(t.t_rq - t.t_start) * 1e-9);
      rb_lat.push_back(static_cast<double>(t.t_rb - t.t_start) * 1e-9);
    } else {
      ++timeouts;
    }
    tracks_.erase(nm);
    early_.erase(nm);
  }
  lk.unlock();
  std::sort(lag.begin(), lag.end());
  const double span = static_cast<double>(last_ready - (t0 + (n ? offset.front() : 0))) * 1e-9;
  out["ready"] = ready;
  out["failed"] = failed;
  out["timeouts"] = timeouts;
  out["offered_rate"] = duration_s > 0 ? static_cast<double>(n) / duration_s : 0.0;
  out["achieved_rate"] = span > 0 ? static_cast<double>(ready) / span : 0.0;
  out["issue_lag_p99_s"] = n ? static_cast<double>(lag[std::min(n - 1, n * 99 / 100)]) * 1e-9 : 0.0;
  out["ready_latency_s"] = lat;
  out["create_latency_s"] = clat;
  out["ns_latency_s"] = ns_lat;
  out["rq_latency_s"] = rq_lat;
  out["rb_latency_s"] = rb_lat;
  out["errors"] = errs;
  out["delete_failures"] = delete_failures_.load();
  return out;
}

void ChurnDriver::approve_batch(const std::vector<std::string>& names,
                                std::chrono::steady_clock::time_point deadline) {
  {
    std::unique_lock<std::mutex> lk(mu_);
    cv_.wait_until(lk, deadline, [&] {
      for (const auto& n : names) {
        const Track& t = tracks_[n];
        if (!t.failed && !t.t_ns) return false;
      }
      return true;
    });
  }
  Value rows = Value::array();
  for (const auto& n : names) rows.push_back(Value::object({{"id_username", n}}));
  Value body = Value::object({{"rows", rows}, {"append", true}});
  http::Headers h;
  h.set("Content-Type", "application/json");
  int64_t t = metrics::now_ns();
  http::Response r = http::fetch("POST", opts_.approve_url, body.dump(), &h);
  if (r.status != 200) throw std::runtime_error("approve: sheet edit failed: " + std::to_string(r.status) + " " + r.body);
  std::lock_guard<std::mutex> lk(mu_);
  for (const auto& n : names) tracks_[n].t_approved = t;
}

int ChurnDriver::remove(const std::vector<std::string>& names) {
  std::vector<std::future<bool>> futs;
  for (const auto& n : names) {
    futs.push_back(pool_->submit([this, n] {
      try {
        admin_->remove(types::UserBootstrap, "", n);
        return true;
      } catch (const kube::ApiError& e) {
        return e.code() == 404;
      } catch (const std::exception&) {
        return false;
      }
    }));
  }
  int failures = 0;
  for (auto& f : futs) failures += f.get() ? 0 : 1;
  std::lock_guard<std::mutex> lk(mu_);
  for (const auto& n : names) early_.erase(n);
  return failures;
}

void ChurnDriver::stop() {
  stop_.cancel();
  for (auto& t : watchers_) {
    if (t.joinable()) t.join();
  }
  watchers_.clear();
}

}  // namespace bgc::bench

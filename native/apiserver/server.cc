#include "apiserver/server.h"

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <functional>
#include <iterator>
#include <mutex>
#include <optional>
#include <regex>
#include <set>
#include <sstream>
#include <thread>
#include <unordered_map>
#include <unordered_set>

#include <openssl/crypto.h>

#include "apiserver/fieldset.h"
#include "core/crypto.h"
#include "core/http.h"
#include "core/json_patch.h"
#include "core/log.h"
#include "core/metrics.h"
#include "core/process.h"
#include "core/stall.h"
#include "core/trace.h"
#include "core/net.h"
#include "core/yaml.h"
#include "crd/schema.h"
#include "kube/leader.h"
#include "kube/quantity.h"
#include "kube/resource.h"

namespace bgc::apiserver {

using json::Value;
using kube::ResourceType;

namespace {

// ---------------------------------------------------------------------------
// Errors as metav1.Status

struct StatusError : std::runtime_error {
  int code;
  std::string reason;
  Value details;
  StatusError(int c, std::string r, const std::string& msg, Value d = {})
      : std::runtime_error(msg), code(c), reason(std::move(r)), details(std::move(d)) {}
};

Value status_body(int code, const std::string& reason, const std::string& message, const Value& details = {}) {
  Value s = Value::object({{"kind", "Status"}, {"apiVersion", "v1"}, {"metadata", Value::object()},
                           {"status", code < 400 ? "Success" : "Failure"}, {"message", message},
                           {"reason", reason}});
  if (!details.is_null()) s["details"] = details;
  s["code"] = code;
  return s;
}

std::string resource_ref(const ResourceType& rt) {
  return rt.group.empty() ? rt.plural : rt.plural + "." + rt.group;
}

StatusError not_found(const ResourceType& rt, const std::string& name) {
  return StatusError(404, "NotFound", resource_ref(rt) + " \"" + name + "\" not found",
                     Value::object({{"name", name}, {"group", rt.group}, {"kind", rt.plural}}));
}

StatusError already_exists(const ResourceType& rt, const std::string& name) {
  return StatusError(409, "AlreadyExists", resource_ref(rt) + " \"" + name + "\" already exists",
                     Value::object({{"name", name}, {"group", rt.group}, {"kind", rt.plural}}));
}

StatusError conflict(const ResourceType& rt, const std::string& name) {
  return StatusError(409, "Conflict",
                     "Operation cannot be fulfilled on " + resource_ref(rt) + " \"" + name +
                         "\": the object has been modified; please apply your changes to the latest version and try again",
                     Value::object({{"name", name}, {"group", rt.group}, {"kind", rt.plural}}));
}

StatusError invalid(const ResourceType& rt, const std::string& name, const std::string& msg) {
  return StatusError(422, "Invalid", rt.kind + "." + rt.group + " \"" + name + "\" is invalid: " + msg,
                     Value::object({{"name", name}, {"group", rt.group}, {"kind", rt.kind}}));
}

std::string now_rfc3339() {
  std::string s = kube::rfc3339_micro_now();
  return s.substr(0, 19) + "Z";
}

bool dns1123_label(const std::string& s) {
  if (s.empty() || s.size() > 63) return false;
  for (size_t i = 0; i < s.size(); ++i) {
    char c = s[i];
    bool ok = (c >= 'a' && c <= 'z') || (c >= '0' && c <= '9') || (c == '-' && i != 0 && i + 1 != s.size());
    if (!ok) return false;
  }
  return true;
}

bool dns1123_subdomain(const std::string& s) {
  if (s.empty() || s.size() > 253) return false;
  size_t start = 0;
  while (true) {
    size_t dot = s.find('.', start);
    std::string part = s.substr(start, dot == std::string::npos ? std::string::npos : dot - start);
    if (!dns1123_label(part)) return false;
    if (dot == std::string::npos) return true;
    start = dot + 1;
  }
}

// ---------------------------------------------------------------------------
// Label selectors

struct Requirement {
  std::string key;
  std::string op;  // = != exists !exists in notin
  std::vector<std::string> values;
};

std::string trim(std::string s) {
  while (!s.empty() && s.front() == ' ') s.erase(0, 1);
  while (!s.empty() && s.back() == ' ') s.pop_back();
  return s;
}

std::vector<Requirement> parse_selector(const std::string& sel) {
  std::vector<Requirement> out;
  // split on commas not inside parentheses
  std::vector<std::string> parts;
  int depth = 0;
  std::string cur;
  for (char c : sel) {
    if (c == '(') ++depth;
    if (c == ')') --depth;
    if (c == ',' && depth == 0) {
      parts.push_back(cur);
      cur.clear();
    } else {
      cur.push_back(c);
    }
  }
  if (!cur.empty()) parts.push_back(cur);
  for (auto p : parts) {
    p = trim(p);
    if (p.empty()) continue;
    Requirement r;
    size_t pos;
    if (p[0] == '!') {
      r.key = trim(p.substr(1));
      r.op = "!exists";
    } else if ((pos = p.find(" notin ")) != std::string::npos || (pos = p.find(" in ")) != std::string::npos) {
      bool notin = p.compare(pos, 7, " notin ") == 0;
      r.key = trim(p.substr(0, pos));
      r.op = notin ? "notin" : "in";
      size_t lp = p.find('('), rp = p.rfind(')');
      if (lp == std::string::npos || rp == std::string::npos) throw StatusError(400, "BadRequest", "invalid selector: " + p);
      std::string inner = p.substr(lp + 1, rp - lp - 1);
      std::stringstream ss(inner);
      std::string v;
      while (std::getline(ss, v, ',')) r.values.push_back(trim(v));
    } else if ((pos = p.find("!=")) != std::string::npos) {
      r.key = trim(p.substr(0, pos));
      r.op = "!=";
      r.values.push_back(trim(p.substr(pos + 2)));
    } else if ((pos = p.find("==")) != std::string::npos) {
      r.key = trim(p.substr(0, pos));
      r.op = "=";
      r.values.push_back(trim(p.substr(pos + 2)));
    } else if ((pos = p.find('=')) != std::string::npos) {
      r.key = trim(p.substr(0, pos));
      r.op = "=";
      r.values.push_back(trim(p.substr(pos + 1)));
    } else {
      r.key = p;
      r.op = "exists";
    }
    out.push_back(r);
  }
  return out;
}

bool selector_matches(const std::vector<Requirement>& reqs, const Value& obj) {
  const Value& labels = obj.get("metadata").get("labels");
  for (const auto& r : reqs) {
    const Value* v = labels.find(r.key);
    bool has = v && v->is_string();
    std::string val = has ? v->as_string() : "";
    if (r.op == "exists" && !has) return false;
    if (r.op == "!exists" && has) return false;
    if (r.op == "=" && (!has || val != r.values[0])) return false;
    if (r.op == "!=" && has && val == r.values[0]) return false;
    if (r.op == "in" && (!has || std::find(r.values.begin(), r.values.end(), val) == r.values.end())) return false;
    if (r.op == "notin" && has && std::find(r.values.begin(), r.values.end(), val) != r.values.end()) return false;
  }
  return true;
}

struct FieldFilter {
  std::string name, ns;
  // kube-lite test extension (a real apiserver rejects the key): only objects whose name
  // starts with this prefix. Used by the bench's per-rank load drivers, so N drivers do not
  // multiply the child-watch fan-out N times; the product binaries never send it.
  std::string name_prefix;
  bool name_ok(std::string_view n) const {
    return (name.empty() || n == name) && (name_prefix.empty() || n.substr(0, name_prefix.size()) == name_prefix);
  }
};

FieldFilter parse_field_selector(const std::string& s) {
  FieldFilter f;
  std::stringstream ss(s);
  std::string part;
  while (std::getline(ss, part, ',')) {
    size_t eq = part.find('=');
    if (eq == std::string::npos) continue;
    std::string k = trim(part.substr(0, eq));
    std::string v = trim(part.substr(part[eq + 1] == '=' ? eq + 2 : eq + 1));
    if (k == "metadata.name") f.name = v;
    else if (k == "metadata.namespace") f.ns = v;
    else if (k == "kube-lite.test/name-prefix") f.name_prefix = v;
  }
  return f;
}

// ---------------------------------------------------------------------------

struct UserInfo {
  std::string username;
  std::string uid;
  std::vector<std::string> groups;
  bool is_admin() const { return std::find(groups.begin(), groups.end(), "system:masters") != groups.end(); }
  Value to_json() const {
    Value g = Value::array();
    for (auto& x : groups) g.push_back(x);
    Value v = Value::object({{"username", username}});
    if (!uid.empty()) v["uid"] = uid;
    v["groups"] = g;
    return v;
  }
};

struct TypeStore;

struct TypeInfo {
  ResourceType rt;
  std::shared_ptr<const Value> schema;  // openAPIV3Schema for CRDs (null for built-ins); atomic swap on CRD update
  bool custom = false;
  std::shared_ptr<TypeStore> store;     // set at registration, never replaced
  std::string key() const { return rt.group + "/" + rt.version + "/" + rt.plural; }
};

struct ManagerEntry {
  std::string operation;  // Apply | Update
  std::string api_version;
  std::string time;
  std::string subresource;
  FieldSet fields;
  bool operator==(const ManagerEntry& o) const {
    return operation == o.operation && fields == o.fields && subresource == o.subresource;
  }
};
using Managers = std::map<std::string, ManagerEntry>;

inline const std::shared_ptr<const Managers>& no_managers() {
  static const std::shared_ptr<const Managers> empty = std::make_shared<const Managers>();
  return empty;
}

struct Stored {
  std::shared_ptr<const Value> obj;
  uint64_t rv = 0;
  // The event line of the commit that stored obj ({"type":"ADDED|MODIFIED","object":<obj>}),
  // while the watch history still holds it: a DELETED event (or a selector transition)
  // reuses that serialization instead of dumping obj again.  Weak, so the store never pins
  // a serialized copy of every live object beyond what history_limit bounds (an object
  // whose commit has been compacted away is serialized anew when deleted).
  std::weak_ptr<const std::string> line;
  // Shared and immutable, like obj: a writer's snapshot of the stored object (taken under
  // the store lock) copies two pointers instead of every manager's field set.
  std::shared_ptr<const Managers> managers = no_managers();
};

// PartialObjectMetadata (meta.k8s.io/v1): what metadata-only clients ask for with
// Accept: application/json;as=PartialObjectMetadata[List];g=meta.k8s.io;v=v1.
bool wants_metadata(const http::Request& req) {
  const std::string* a = req.headers.get("Accept");
  return a && a->find("as=PartialObjectMetadata") != std::string::npos;
}

void dump_partial_metadata(const Value& obj, std::string& out) {
  out += "{\"kind\":\"PartialObjectMetadata\",\"apiVersion\":\"meta.k8s.io/v1\",\"metadata\":";
  obj.get("metadata").dump_to(out);
  out += "}";
}

// {"type":T,"object":O}\n -> {"type":T,"object":<PartialObjectMetadata of O>}\n, from the
// serialized line (no re-parse of the object).
std::string partial_metadata_line(const std::string& line) {
  std::string_view body(line);
  while (!body.empty() && (body.back() == '\n' || body.back() == '\r')) body.remove_suffix(1);
  const std::string_view type = json::raw_member(body, "type");
  const std::string_view md = json::raw_member(json::raw_member(body, "object"), "metadata");
  std::string out;
  out.reserve(md.size() + 128);
  out += "{\"type\":";
  out.append(type.data(), type.size());
  out += ",\"object\":{\"kind\":\"PartialObjectMetadata\",\"apiVersion\":\"meta.k8s.io/v1\",\"metadata\":";
  if (md.empty()) out += "{}";
  else out.append(md.data(), md.size());
  out += "}}\n";
  return out;
}

// How one watch sees one event (EventRec::line_as).  A label-selector watch sees an update
// that moves the object into its selector as ADDED and one that moves it out as DELETED
// (carrying the previous object at the event's resourceVersion), as the kube-apiserver's
// watch cache does (cacheWatcher.convertToWatchEvent); every other event as it is.
enum class View : uint8_t { AsIs, Added, Deleted };

struct EventRec {
  uint64_t rv;
  std::string type_key;
  std::string ns;
  // Only what a resuming watch filters on ({"metadata":{"name","labels"}}), not the
  // object: the watch cache must not pin every old version's full tree in memory.
  std::shared_ptr<const Value> meta;
  std::shared_ptr<const std::string> line;  // {"type":..,"object":..}\n
  // Updates that changed the object's labels (selector transitions possible): the previous
  // version's filter view and its committed event line, and the transition lines built from
  // them on first use.  Null for every other event (most of them).
  struct Transitions {
    std::shared_ptr<const Value> prev_meta;
    std::shared_ptr<const std::string> prev_line;
    std::once_flag added_once, deleted_once;
    std::string added, added_meta, deleted, deleted_meta;
  };
  std::unique_ptr<Transitions> tr;
  // The PartialObjectMetadata form, built once on first use by a metadata-only watch.
  const std::string& metadata_line() const {
    std::call_once(meta_once_, [this] { meta_line_ = partial_metadata_line(*line); });
    return meta_line_;
  }
  // The line a watch with this view receives (transition forms built once, on first use).
  const std::string& line_as(View v, bool meta_only) const {
    if (v == View::AsIs || !tr) return meta_only ? metadata_line() : *line;
    Transitions& t = *tr;
    if (v == View::Added) {
      std::call_once(t.added_once, [&] {
        t.added = retyped_line(*line, "ADDED");
        t.added_meta = partial_metadata_line(t.added);
      });
      return meta_only ? t.added_meta : t.added;
    }
    std::call_once(t.deleted_once, [&] {
      t.deleted = deleted_from_prev();
      t.deleted_meta = partial_metadata_line(t.deleted);
    });
    return meta_only ? t.deleted_meta : t.deleted;
  }

 private:
  // {"type":T,...} -> {"type":<type>,...}
  static std::string retyped_line(const std::string& l, const char* type) {
    const std::string_view t = json::raw_member(l, "type");
    std::string out;
    if (t.empty()) return l;
    out.reserve(l.size() + 8);
    out.append(l, 0, static_cast<size_t>(t.data() - l.data()));
    out += '"';
    out += type;
    out += '"';
    out.append(t.data() + t.size(), l.data() + l.size());
    return out;
  }
  // DELETED with the previous object, its resourceVersion replaced by this event's
  std::string deleted_from_prev() const {
    std::string_view prev(*tr->prev_line);
    while (!prev.empty() && (prev.back() == '\n' || prev.back() == '\r')) prev.remove_suffix(1);
    const std::string_view obj = json::raw_member(prev, "object");
    const std::string_view old_rv = json::raw_member(json::raw_member(obj, "metadata"), "resourceVersion");
    const std::string_view new_rv =
        json::raw_member(json::raw_member(json::raw_member(*line, "object"), "metadata"), "resourceVersion");
    std::string out = "{\"type\":\"DELETED\",\"object\":";
    if (old_rv.empty()) {
      out.append(obj.data(), obj.size());
    } else {
      out.append(obj.data(), static_cast<size_t>(old_rv.data() - obj.data()));
      out.append(new_rv.data(), new_rv.size());
      out.append(old_rv.data() + old_rv.size(), obj.data() + obj.size());
    }
    out += "}\n";
    return out;
  }
  mutable std::once_flag meta_once_;
  mutable std::string meta_line_;
};

struct QueuedEvent {
  std::shared_ptr<const EventRec> e;
  View view = View::AsIs;
};

// {"metadata":{"name":..,"labels":..}} of an object: the fields watch filters read.
std::shared_ptr<const Value> filter_view(const Value& obj) {
  const Value& m = obj.get("metadata");
  Value meta = Value::object({{"name", m.get("name")}});
  if (m.contains("labels")) meta["labels"] = m.get("labels");
  return std::make_shared<const Value>(Value::object({{"metadata", std::move(meta)}}));
}

struct WatchSub {
  std::string type_key;
  std::string ns;
  std::vector<Requirement> sel;
  FieldFilter fields;
  // q/closed/overflow are guarded by m (not the store mutex): a watch stream waking up for
  // an event never contends with writers. Lock order: store mutex -> m.
  std::mutex m;
  std::condition_variable cv;
  std::deque<QueuedEvent> q;
  bool closed = false;
  bool overflow = false;

  void close() {
    {
      std::lock_guard<std::mutex> g(m);
      closed = true;
    }
    cv.notify_one();
  }
};

// Store lock.  Default: one mutex (futex wake-one) for reads and commits alike.  The
// reader/writer lock used before (writer-preferring, since glibc's default starves commits
// under a steady GET/LIST load) woke every waiting reader at each commit's unlock: at 800
// creates in flight its wake-up herd cost more than the read parallelism gained
// (profiles/archive/kl_store_lock_r2/: N=8 +63 % CR/s, kube-lite CPU per CR 4.2 -> 2.2 ms with the
// mutex; N=1 +17 %).  BGC_KL_RWLOCK=writer|reader selects the rwlock variants.
class RwLock {
 public:
  RwLock() {
    const char* kind = std::getenv("BGC_KL_RWLOCK");  // unset/"mutex": one mutex; "writer" / "reader": rwlock
    mutex_only_ = !kind || (std::string(kind) != "writer" && std::string(kind) != "reader");
    pthread_rwlockattr_t a;
    pthread_rwlockattr_init(&a);
    pthread_rwlockattr_setkind_np(&a, kind && std::string(kind) == "reader" ? PTHREAD_RWLOCK_PREFER_READER_NP
                                                                           : PTHREAD_RWLOCK_PREFER_WRITER_NONRECURSIVE_NP);
    pthread_rwlock_init(&l_, &a);
    pthread_rwlockattr_destroy(&a);
  }
  ~RwLock() { pthread_rwlock_destroy(&l_); }
  RwLock(const RwLock&) = delete;
  RwLock& operator=(const RwLock&) = delete;
  void lock() {
    if (mutex_only_) m_.lock();
    else pthread_rwlock_wrlock(&l_);
  }
  bool try_lock() { return mutex_only_ ? m_.try_lock() : pthread_rwlock_trywrlock(&l_) == 0; }
  void unlock() {
    if (mutex_only_) m_.unlock();
    else pthread_rwlock_unlock(&l_);
  }
  void lock_shared() {
    if (mutex_only_) m_.lock();
    else pthread_rwlock_rdlock(&l_);
  }
  bool try_lock_shared() { return mutex_only_ ? m_.try_lock() : pthread_rwlock_tryrdlock(&l_) == 0; }
  void unlock_shared() { unlock(); }

 private:
  pthread_rwlock_t l_;
  std::mutex m_;
  bool mutex_only_ = false;
};

// Watch wake-ups are deferred until the exclusive store lock is released (a futex wake per
// subscriber inside the critical section would stretch every commit).
thread_local std::vector<std::shared_ptr<WatchSub>> t_pending_wakeups;
// History records compacted away under a lock: their lines are freed after it is released.
thread_local std::vector<std::shared_ptr<const EventRec>> t_retired_events;

inline void flush_watch_wakeups() {
  for (auto& w : t_pending_wakeups) w->cv.notify_one();
  t_pending_wakeups.clear();
  t_retired_events.clear();
}

// Store-lock accounting (exported in /_kl/stats): exclusive hold time bounds kube-lite's
// commit throughput (commits/s <= 1 / mean exclusive hold).
struct LockStats {
  std::atomic<uint64_t> acquisitions{0}, shared{0}, contended{0}, wait_ns{0}, hold_ns{0};
};

class StoreLock {  // exclusive
 public:
  // `also`: a second account of the same acquisition (a type's seq lock: its own stats
  // and the type's total)
  StoreLock(RwLock& m, LockStats& st, LockStats* also = nullptr) : m_(m), st_(st), also_(also) {
    if (!m_.try_lock()) {
      int64_t t0 = metrics::now_ns();
      m_.lock();
      const auto waited = static_cast<uint64_t>(metrics::now_ns() - t0);
      st_.contended.fetch_add(1, std::memory_order_relaxed);
      st_.wait_ns.fetch_add(waited, std::memory_order_relaxed);
      if (also_) {
        also_->contended.fetch_add(1, std::memory_order_relaxed);
        also_->wait_ns.fetch_add(waited, std::memory_order_relaxed);
      }
    }
    t_acq_ = metrics::now_ns();
  }
  ~StoreLock() {
    const auto held = static_cast<uint64_t>(metrics::now_ns() - t_acq_);
    st_.acquisitions.fetch_add(1, std::memory_order_relaxed);
    st_.hold_ns.fetch_add(held, std::memory_order_relaxed);
    if (also_) {
      also_->acquisitions.fetch_add(1, std::memory_order_relaxed);
      also_->hold_ns.fetch_add(held, std::memory_order_relaxed);
    }
    m_.unlock();
    flush_watch_wakeups();
  }
  StoreLock(const StoreLock&) = delete;
  StoreLock& operator=(const StoreLock&) = delete;

 private:
  RwLock& m_;
  LockStats& st_;
  LockStats* also_;
  int64_t t_acq_ = 0;
};

class SharedStoreLock {
 public:
  SharedStoreLock(RwLock& m, LockStats& st) : m_(m) {
    if (!m_.try_lock_shared()) {
      int64_t t0 = metrics::now_ns();
      m_.lock_shared();
      st.contended.fetch_add(1, std::memory_order_relaxed);
      st.wait_ns.fetch_add(static_cast<uint64_t>(metrics::now_ns() - t0), std::memory_order_relaxed);
    }
    st.shared.fetch_add(1, std::memory_order_relaxed);
  }
  ~SharedStoreLock() { m_.unlock_shared(); }
  SharedStoreLock(const SharedStoreLock&) = delete;
  SharedStoreLock& operator=(const SharedStoreLock&) = delete;

 private:
  RwLock& m_;
};

// Per-resource-type storage (like the apiserver's per-resource storage and watch cache):
// its objects, event history and watchers, so commits to different types never serialize
// on each other.  Within a type:
//  * objects live in Options::store_shards key-hashed shards, each with its own lock:
//    reads and commits of different objects proceed in parallel (a commit's stored-version
//    check and its map update run under its object's shard only; the webhook, merge and
//    validation before it under no lock).  One shard is a single lock per type;
//  * `seq` orders the type's events: a commit, holding its object's shard exclusively,
//    takes seq only to assign the resourceVersion and append the event to the history
//    and to the watchers' queues.  Lock order: shard -> seq -> watches_mu -> WatchSub::m.
//  * a whole-type read (LIST, a watch's initial snapshot) holds every shard (AllShards),
//    so no commit of the type is in flight while it reads; a watch resuming from a
//    resourceVersion holds seq while it replays the history and registers.
struct TypeStore {
  struct Shard {
    RwLock mu;
    std::unordered_map<std::string, Stored> objs;  // obj key -> stored (guarded by mu)
  };
  // A fixed array of n shards (RwLock is neither movable nor copyable), iterable.
  class Shards {
   public:
    explicit Shards(size_t n) : n_(std::max<size_t>(1, n)), p_(new Shard[n_]) {}
    Shard* begin() { return p_.get(); }
    Shard* end() { return p_.get() + n_; }
    std::reverse_iterator<Shard*> rbegin() { return std::reverse_iterator<Shard*>(end()); }
    std::reverse_iterator<Shard*> rend() { return std::reverse_iterator<Shard*>(begin()); }
    size_t size() const { return n_; }
    Shard& operator[](size_t i) { return p_[i]; }

   private:
    size_t n_;
    std::unique_ptr<Shard[]> p_;
  };
  explicit TypeStore(size_t n_shards) : shards(n_shards) {}
  Shards shards;
  Shard& shard(const std::string& key) {
    return shards.size() == 1 ? shards[0] : shards[std::hash<std::string>{}(key) % shards.size()];
  }
  RwLock seq;
  std::atomic<uint64_t> version{0};                          // bumped by every commit/erase (under seq)
  LockStats stats;                                           // the shard locks
  LockStats seq_stats;                                       // seq (the type's commit order)
  std::deque<std::shared_ptr<const EventRec>> history;       // rv-ordered (appended under seq)
  uint64_t compacted_rv = 0;                                 // resumes from rv < compacted_rv get 410
  std::mutex watches_mu;                                     // lock order: seq -> watches_mu -> WatchSub::m
  std::set<std::shared_ptr<WatchSub>> watches;
};

// Every shard of a type, in index order (the same order commits can never hold two of).
class AllShards {
 public:
  AllShards(TypeStore& ts, bool exclusive) : ts_(ts), exclusive_(exclusive) {
    for (auto& sh : ts_.shards) {
      if (exclusive_) {
        if (!sh.mu.try_lock()) {
          const int64_t t0 = metrics::now_ns();
          sh.mu.lock();
          ts_.stats.contended.fetch_add(1, std::memory_order_relaxed);
          ts_.stats.wait_ns.fetch_add(static_cast<uint64_t>(metrics::now_ns() - t0), std::memory_order_relaxed);
        }
      } else if (!sh.mu.try_lock_shared()) {
        const int64_t t0 = metrics::now_ns();
        sh.mu.lock_shared();
        ts_.stats.contended.fetch_add(1, std::memory_order_relaxed);
        ts_.stats.wait_ns.fetch_add(static_cast<uint64_t>(metrics::now_ns() - t0), std::memory_order_relaxed);
      }
    }
    ts_.stats.acquisitions.fetch_add(1, std::memory_order_relaxed);
  }
  ~AllShards() {
    for (auto it = ts_.shards.rbegin(); it != ts_.shards.rend(); ++it) {
      if (exclusive_) it->mu.unlock();
      else it->mu.unlock_shared();
    }
    flush_watch_wakeups();
  }
  AllShards(const AllShards&) = delete;
  AllShards& operator=(const AllShards&) = delete;

 private:
  TypeStore& ts_;
  bool exclusive_;
};

struct FaultRule {
  std::string method;  // empty = any
  std::regex path;
  std::string path_src;
  int status = 0;
  int retry_after_s = -1;  // >= 0: send a Retry-After header (429 / 503 throttling)
  int delay_ms = 0;
  // served as usual, then the response is held this long ("delay_response_ms"): the write
  // is committed and its watch event delivered before the client has its answer
  int hold_ms = 0;
  int remaining = -1;  // -1 = unlimited
  bool reset = false;  // drop the connection without a response
  std::string message;
};

struct ParsedPath {
  TypeInfo* ti = nullptr;
  std::string ns;
  std::string name;
  std::string sub;
  bool collection = false;
};

// Per-request trace context (core/trace.h), on the thread that serves the request: set by
// Impl::handle while the bench has tracing armed, read by write()/do_delete to mark the
// webhook call and the commit.  Empty when not tracing.
thread_local std::string t_trace_tag;   // "<plural>[/sub].<METHOD>.<field manager>"
thread_local std::string t_trace_name;  // the object's name (a tenant's, for every child)

void trace_step(const std::string& name, const char* step) {
  if (!t_trace_tag.empty()) trace::mark(name, t_trace_tag + step);
}

struct WriteResult {
  std::shared_ptr<const Value> obj;
  int code = 200;
  // The committed watch-event line, whose "object" member is exactly the response body:
  // a write serializes its object once (for the event) and answers with a view into it.
  std::shared_ptr<const std::string> line;
  std::string_view body() const {
    static const std::string kPrefixEnd = ",\"object\":";
    if (!line) return {};
    size_t at = line->find(kPrefixEnd);
    if (at == std::string::npos || line->size() < at + kPrefixEnd.size() + 2) return {};
    at += kPrefixEnd.size();
    return std::string_view(*line).substr(at, line->size() - at - 2);  // drop the closing "}\n"
  }
};

std::string obj_key(const ResourceType& rt, const std::string& ns, const std::string& name) { return rt.key(ns, name); }

}  // namespace

// ===========================================================================

struct ApiServer::Impl {
  Options opts;
  std::unique_ptr<http::Server> server;

  // Lock order: one TypeStore::mu at a time -> types_mu / index_mu -> TypeStore::watches_mu
  // -> WatchSub::m. Nothing that holds types_mu or index_mu acquires a TypeStore lock.
  RwLock types_mu;                        // guards `types` (CRD registration is the only writer)
  std::map<std::string, TypeInfo> types;  // key() -> info; nodes are never erased (stable pointers)
  std::atomic<uint64_t> rv{1000};         // global resourceVersion; fetched under the owning type's exclusive lock
  std::mutex index_mu;                    // guards the three indexes below
  std::unordered_map<std::string, std::pair<std::string, std::string>> by_uid;      // uid -> (type key, obj key)
  // Secondary indexes so garbage collection and namespace cascades touch only the
  // affected objects (O(dependents), not O(all objects)).
  using Ref = std::pair<std::string, std::string>;  // (type key, obj key)
  struct RefHash {
    size_t operator()(const Ref& r) const { return std::hash<std::string>{}(r.first) * 31 + std::hash<std::string>{}(r.second); }
  };
  std::unordered_map<std::string, std::unordered_set<Ref, RefHash>> by_owner;      // owner uid -> dependents
  std::unordered_map<std::string, std::unordered_set<Ref, RefHash>> by_namespace;  // namespace -> objects

  // Background garbage collector (the apiserver's GC controller does cascading deletion
  // asynchronously too): deletions enqueue owner uids / namespace names.
  struct GcItem {
    bool is_namespace = false;
    std::string id;  // owner uid or namespace name
    bool finish_namespace = false;  // then remove the (Terminating) namespace itself
  };
  std::mutex gc_mu;
  std::condition_variable gc_cv;
  std::deque<GcItem> gc_queue;
  bool gc_stop = false;
  std::atomic<uint64_t> gc_collected{0};
  std::vector<std::thread> gc_threads;

  std::unordered_map<std::string, UserInfo> tokens;

  std::mutex fault_mu;
  std::vector<FaultRule> faults;

  // Paginated LIST snapshots (continue tokens).
  struct ListSnapshot {
    uint64_t rv = 0;
    std::vector<std::shared_ptr<const Value>> items;
    std::chrono::steady_clock::time_point expires;
  };
  std::mutex list_mu;
  std::map<uint64_t, ListSnapshot> list_snapshots;
  uint64_t next_list_id = 1;
  std::atomic<uint64_t> list_pages{0};

  // resourceVersion <-> wire string (decimal, or opaque "kl.<base36>" with --opaque-rv)
  static constexpr uint64_t kRvMask = 0x5bd1e9955bd1e995ULL;
  std::string rv_str(uint64_t v) const {
    if (!opts.opaque_rv) return std::to_string(v);
    static const char* digits = "0123456789abcdefghijklmnopqrstuvwxyz";
    uint64_t x = v ^ kRvMask;
    std::string out;
    do {
      out.insert(out.begin(), digits[x % 36]);
      x /= 36;
    } while (x);
    return "kl." + out;
  }
  // false when the string is not a resourceVersion this server issued
  bool parse_rv(const std::string& s, uint64_t* v) const {
    if (!opts.opaque_rv) {
      if (s.empty() || s.find_first_not_of("0123456789") != std::string::npos) return false;
      *v = std::strtoull(s.c_str(), nullptr, 10);
      return true;
    }
    if (s.rfind("kl.", 0) != 0 || s.size() < 4) return false;
    uint64_t x = 0;
    for (size_t i = 3; i < s.size(); ++i) {
      const char c = s[i];
      int d = c >= '0' && c <= '9' ? c - '0' : c >= 'a' && c <= 'z' ? c - 'a' + 10 : -1;
      if (d < 0) return false;
      x = x * 36 + static_cast<uint64_t>(d);
    }
    *v = x ^ kRvMask;
    return true;
  }

  std::mutex hook_mu;
  struct FastHook {
    std::shared_ptr<const Value> cfg;
    std::shared_ptr<http::Client> client;
    std::string path;
  };
  std::map<const Value*, FastHook> hook_fast;  // guarded by hook_mu
  std::map<std::string, std::shared_ptr<http::Client>> hook_clients;
  // webhook transport for new clients (--webhook-http2; switchable at run time through
  // POST /_kl/webhook-protocol so one bench run can time both)
  std::atomic<bool> webhook_h2{false};
  // storage commit latency (Options::write_latency_us), switchable at run time through
  // POST /_kl/write-latency-us so one bench run can time several etcd models
  std::atomic<int64_t> write_latency_us{0};
  // Options::watch_coalesce_us, switchable at run time through POST /_kl/watch-coalesce-us:
  // the bench's open-loop windows time latency without the coalescing hold, its closed-loop
  // phases keep the throughput it buys (profiles/r6_coalesce_ab/)
  std::atomic<int> watch_coalesce_us{0};

  std::atomic<uint64_t> requests{0};
  std::atomic<uint64_t> faults_hit{0};
  LockStats types_stats;  // types_mu accounting

  explicit Impl(Options o) : opts(std::move(o)) {
    if (const char* e = std::getenv("BGC_KL_STORE_SHARDS"); e && *e) opts.store_shards = std::max(1, std::atoi(e));
    watch_coalesce_us = opts.watch_coalesce_us;
    if (const char* e = std::getenv("BGC_KL_H2_CALLER_READS"); e && *e) opts.webhook_h2_caller_reads = std::string(e) != "0";
    webhook_h2 = opts.webhook_http2;
    write_latency_us = opts.write_latency_us;
    for (const ResourceType* rt : kube::types::builtin()) {
      TypeInfo ti;
      ti.rt = *rt;
      ti.store = std::make_shared<TypeStore>(opts.store_shards);
      types[ti.key()] = ti;
    }
    if (!opts.token_file.empty()) load_tokens(opts.token_file);
    // the namespaces every cluster starts with (the apiserver's system namespace controller)
    const TypeInfo& ns_ti = types.at(kube::types::Namespace.group + "/" + kube::types::Namespace.version + "/" +
                                     kube::types::Namespace.plural);
    for (const char* name : {"default", "kube-system", "kube-public", "kube-node-lease"}) {
      const uint64_t v = ++rv;
      Value ns = Value::object(
          {{"apiVersion", "v1"}, {"kind", "Namespace"},
           {"metadata", Value::object({{"name", name}, {"uid", crypto::uuid_v4()}, {"creationTimestamp", now_rfc3339()},
                                       {"resourceVersion", rv_str(v)}})},
           {"spec", Value::object({{"finalizers", Value::array({Value("kubernetes")})}})},
           {"status", Value::object({{"phase", "Active"}})}});
      Stored st;
      st.obj = std::make_shared<const Value>(std::move(ns));
      st.rv = v;
      ns_ti.store->shard(obj_key(ns_ti.rt, "", name)).objs[obj_key(ns_ti.rt, "", name)] = std::move(st);
    }
    for (int i = 0; i < std::max(1, opts.gc_workers); ++i) gc_threads.emplace_back([this] {
      gc_loop();
      OPENSSL_thread_stop();  // per-thread OpenSSL state (uuid_v4's DRBG, error queue)
    });
  }

  ~Impl() {
    {
      std::lock_guard<std::mutex> g(gc_mu);
      gc_stop = true;
    }
    gc_cv.notify_all();
    for (auto& t : gc_threads) t.join();
  }

  template <typename F>
  void for_each_store(F f) {
    std::vector<std::pair<std::string, std::shared_ptr<TypeStore>>> stores;
    {
      SharedStoreLock lk(types_mu, types_stats);
      for (auto& [k, ti] : types) stores.emplace_back(k, ti.store);
    }
    for (auto& [k, st] : stores) f(k, *st);
  }

  TypeInfo* type_by_key(const std::string& key) {
    SharedStoreLock lk(types_mu, types_stats);
    auto it = types.find(key);
    return it == types.end() ? nullptr : &it->second;
  }

  void load_tokens(const std::string& path) {
    std::stringstream ss(net::read_file(path));
    std::string line;
    while (std::getline(ss, line)) {
      if (line.empty() || line[0] == '#') continue;
      std::vector<std::string> cols;
      std::string cur;
      bool q = false;
      for (char c : line) {
        if (c == '"') {
          q = !q;
          continue;
        }
        if (c == ',' && !q) {
          cols.push_back(cur);
          cur.clear();
          continue;
        }
        cur.push_back(c);
      }
      cols.push_back(cur);
      if (cols.size() < 2) continue;
      UserInfo u;
      u.username = cols[1];
      if (cols.size() > 2) u.uid = cols[2];
      if (cols.size() > 3 && !cols[3].empty()) {
        std::stringstream gs(cols[3]);
        std::string g;
        while (std::getline(gs, g, ',')) u.groups.push_back(g);
      }
      u.groups.push_back("system:authenticated");
      tokens[cols[0]] = u;
    }
  }

  // ---------------------------------------------------------------- auth
  UserInfo authenticate(const http::Request& req) {
    UserInfo u;
    std::string auth = req.headers.get_or("Authorization");
    if (auth.rfind("Bearer ", 0) == 0) {
      auto it = tokens.find(auth.substr(7));
      if (it == tokens.end()) throw StatusError(401, "Unauthorized", "Unauthorized");
      u = it->second;
    } else if (!req.peer_cn.empty()) {
      // x509 authenticator: CN is the user name, each O a group
      u.username = req.peer_cn;
      u.groups = req.peer_orgs;
      u.groups.push_back("system:authenticated");
    } else if (opts.anonymous_admin) {
      u.username = "system:admin";
      u.groups = {"system:masters", "system:authenticated"};
    } else {
      throw StatusError(401, "Unauthorized", "Unauthorized");
    }
    if (const std::string* imp = req.headers.get("Impersonate-User")) {
      if (!u.is_admin()) {
        throw StatusError(403, "Forbidden", "users \"" + *imp + "\" is forbidden: User \"" + u.username +
                                                "\" cannot impersonate resource \"users\" in API group \"\" at the cluster scope");
      }
      UserInfo imp_u;
      imp_u.username = *imp;
      for (const auto& kv : req.headers.items()) {
        std::string lk = kv.first;
        for (auto& c : lk) c = static_cast<char>(std::tolower(static_cast<unsigned char>(c)));
        if (lk == "impersonate-group") {
          // one header per group per the spec; comma-joined values are split too
          // because common HTTP client libraries fold repeated headers.
          std::stringstream gs(kv.second);
          std::string g;
          while (std::getline(gs, g, ',')) {
            if (!trim(g).empty()) imp_u.groups.push_back(trim(g));
          }
        }
      }
      imp_u.groups.push_back("system:authenticated");
      u = imp_u;
    }
    return u;
  }

  // ---------------------------------------------------------------- paths
  TypeInfo* find_type(const std::string& group, const std::string& version, const std::string& plural) {
    auto it = types.find(group + "/" + version + "/" + plural);
    return it == types.end() ? nullptr : &it->second;
  }

  // Returns false for non-resource (discovery) paths.
  bool parse_path(const std::string& path, ParsedPath& out, std::string& group, std::string& version,
                  std::vector<std::string>& rest) {
    std::vector<std::string> segs;
    std::stringstream ss(path);
    std::string s;
    while (std::getline(ss, s, '/')) {
      if (!s.empty()) segs.push_back(s);
    }
    size_t i = 0;
    if (segs.size() >= 2 && segs[0] == "api") {
      group = "";
      version = segs[1];
      i = 2;
    } else if (segs.size() >= 3 && segs[0] == "apis") {
      group = segs[1];
      version = segs[2];
      i = 3;
    } else {
      return false;
    }
    rest.assign(segs.begin() + static_cast<long>(i), segs.end());
    if (rest.empty()) return false;
    SharedStoreLock lk(types_mu, types_stats);
    if (rest[0] == "namespaces" && rest.size() >= 3) {
      TypeInfo* ti = find_type(group, version, rest[2]);
      if (ti && ti->rt.namespaced) {
        out.ti = ti;
        out.ns = rest[1];
        out.collection = rest.size() == 3;
        if (rest.size() >= 4) out.name = rest[3];
        if (rest.size() >= 5) out.sub = rest[4];
        return true;
      }
    }
    TypeInfo* ti = find_type(group, version, rest[0]);
    if (!ti) throw StatusError(404, "NotFound", "the server could not find the requested resource");
    out.ti = ti;
    out.collection = rest.size() == 1;
    if (rest.size() >= 2) out.name = rest[1];
    if (rest.size() >= 3) out.sub = rest[2];
    return true;
  }

  // ---------------------------------------------------------------- events
  // Work moved out of the exclusive section (see prepare_commit).
  struct PreparedEvent {
    std::string head, tail;  // event line = head + rv digits + tail
    bool ok = false;
    // built before the exclusive section: the resuming-watch filter view and the event
    // record (its line is filled in under the lock)
    std::shared_ptr<const Value> filter;
    std::shared_ptr<EventRec> rec;
  };

  // Appends one event to the type's history and to its watchers' queues.  Caller holds
  // ti.store->seq.  `filter` is the event object's {"metadata":{"name","labels"}} view,
  // which is all a watch filters on.
  std::shared_ptr<const std::string> emit_locked(const TypeInfo& ti, const std::string& ns, uint64_t ev_rv,
                                                 std::string line, std::shared_ptr<const Value> filter,
                                                 std::shared_ptr<EventRec> rec) {
    TypeStore& st = *ti.store;
    st.version.fetch_add(1, std::memory_order_release);
    if (!rec) rec = std::make_shared<EventRec>();
    rec->rv = ev_rv;
    rec->type_key = ti.key();
    rec->ns = ns;
    rec->meta = std::move(filter);
    rec->line = std::make_shared<const std::string>(std::move(line));
    st.history.push_back(rec);
    while (st.history.size() > opts.history_limit) {
      st.compacted_rv = st.history.front()->rv;
      t_retired_events.push_back(std::move(st.history.front()));  // freed after the lock
      st.history.pop_front();
    }
    const std::string& name = rec->meta->get("metadata").get_string("name");
    std::lock_guard<std::mutex> wg(st.watches_mu);
    for (const auto& w : st.watches) {
      if (!w->ns.empty() && w->ns != ns) continue;
      if (!w->fields.name_ok(name)) continue;
      View view;
      if (!view_for(w->sel, *rec, &view)) continue;
      {
        std::lock_guard<std::mutex> g(w->m);
        if (w->q.size() > 100000) w->overflow = true;
        else w->q.push_back({rec, view});
      }
      t_pending_wakeups.push_back(w);
    }
    return rec->line;
  }

  // Whether a watch with label selector `sel` receives `e`, and as what.
  static bool view_for(const std::vector<Requirement>& sel, const EventRec& e, View* view) {
    *view = View::AsIs;
    if (sel.empty()) return true;
    const bool now_in = selector_matches(sel, *e.meta);
    if (!e.tr) return now_in;
    const bool was_in = selector_matches(sel, *e.tr->prev_meta);
    if (now_in && !was_in) *view = View::Added;
    else if (!now_in && was_in) *view = View::Deleted;
    return now_in || was_in;
  }

  // ---------------------------------------------------------------- webhooks
  struct HookMatch {
    std::string name;
    std::shared_ptr<const Value> cfg;  // keeps `hook` alive (stored objects are immutable)
    const Value* hook;
  };
  std::mutex hook_match_mu;                    // matching_webhooks' cache
  uint64_t hook_match_version = ~uint64_t{0};  // MWC store version the cache is for
  std::unordered_map<std::string, std::vector<HookMatch>> hook_match_cache;

  // The hooks a request triggers, cached per (type, subresource, operation) for one version
  // of the MutatingWebhookConfigurations: every UserBootstrap write asks, and scanning the
  // configurations under all their shard locks each time serialized the writers.
  std::vector<HookMatch> matching_webhooks(const TypeInfo& ti, const std::string& sub, const std::string& op) {
    TypeInfo* mwc = type_by_key(kube::types::MutatingWebhookConfiguration.group + "/v1/mutatingwebhookconfigurations");
    if (!mwc) return {};
    const std::string cache_key = ti.key() + "|" + sub + "|" + op;
    {
      std::lock_guard<std::mutex> g(hook_match_mu);
      if (hook_match_version == mwc->store->version.load(std::memory_order_acquire)) {
        auto it = hook_match_cache.find(cache_key);
        if (it != hook_match_cache.end()) return it->second;
      }
    }
    std::vector<HookMatch> out;
    AllShards lk(*mwc->store, false);
    const uint64_t version = mwc->store->version.load(std::memory_order_acquire);  // no commit in flight
    std::string res = ti.rt.plural + (sub.empty() ? "" : "/" + sub);
    for (auto& sh : mwc->store->shards)
    for (auto& kv : sh.objs) {
      for (const auto& hook : kv.second.obj->get("webhooks").items()) {
        for (const auto& rule : hook.get("rules").items()) {
          auto contains = [](const Value& arr, const std::string& v) {
            for (const auto& x : arr.items()) {
              if (x.is_string() && (x.as_string() == "*" || x.as_string() == v)) return true;
            }
            return false;
          };
          bool res_ok = false;
          for (const auto& r : rule.get("resources").items()) {
            std::string rs = r.as_string();
            if (rs == res || rs == "*/*" || (rs == "*" && sub.empty()) ||
                (sub.size() && rs == "*/" + sub) || (rs == ti.rt.plural + "/*")) {
              res_ok = true;
            }
          }
          if (contains(rule.get("apiGroups"), ti.rt.group) && contains(rule.get("apiVersions"), ti.rt.version) &&
              contains(rule.get("operations"), op) && res_ok) {
            out.push_back({hook.get_string("name"), kv.second.obj, &hook});
            break;
          }
        }
      }
    }
    {
      std::lock_guard<std::mutex> g(hook_match_mu);
      if (hook_match_version != version) {
        hook_match_cache.clear();
        hook_match_version = version;
      }
      hook_match_cache[cache_key] = out;
    }
    return out;
  }

  // Per-hook client cache keyed by the hook's address inside its (immutable, kept-alive)
  // configuration object: no re-hashing of the caBundle per call.
  std::shared_ptr<http::Client> hook_client(const HookMatch& hm, std::string& path_out) {
    {
      std::lock_guard<std::mutex> lk(hook_mu);
      auto it = hook_fast.find(hm.hook);
      if (it != hook_fast.end()) {
        path_out = it->second.path;
        return it->second.client;
      }
    }
    auto c = hook_client_slow(*hm.hook, path_out);
    std::lock_guard<std::mutex> lk(hook_mu);
    if (hook_fast.size() > 256) hook_fast.clear();
    hook_fast[hm.hook] = {hm.cfg, c, path_out};
    return c;
  }

  std::shared_ptr<http::Client> hook_client_slow(const Value& hook, std::string& path_out) {
    const Value& cc = hook.get("clientConfig");
    std::string ca = cc.get_string("caBundle");
    std::string base, server_name;
    if (cc.get("url").is_string()) {
      http::Url u = http::parse_url(cc.get_string("url"));
      base = u.scheme + "://" + u.host + ":" + std::to_string(u.port);
      path_out = u.path.empty() ? "/" : u.path;
    } else {
      const Value& svc = cc.get("service");
      std::string ns = svc.get_string("namespace"), name = svc.get_string("name");
      int port = svc.get("port").is_int() ? static_cast<int>(svc.get("port").as_int()) : 443;
      path_out = svc.get_string("path", "/");
      server_name = name + "." + ns + ".svc";
      auto ov = opts.service_overrides.find(ns + "/" + name);
      std::string hostport = ov != opts.service_overrides.end() ? ov->second : server_name + ":" + std::to_string(port);
      base = "https://" + hostport;
    }
    std::string key = base + "|" + server_name + "|" + crypto::sha256_hex(ca);
    std::lock_guard<std::mutex> lk(hook_mu);
    auto it = hook_clients.find(key);
    if (it != hook_clients.end()) return it->second;
    http::ClientOptions o;
    o.base_url = base;
    o.tls_server_name = server_name;
    o.http2 = webhook_h2.load();
    o.h2_connections = opts.webhook_h2_connections;
    o.h2_caller_reads = opts.webhook_h2_caller_reads;
    if (base.rfind("https", 0) == 0) {
      o.tls = net::TlsContext::client(ca.empty() ? "" : crypto::base64_decode(ca), false);
    }
    auto c = std::make_shared<http::Client>(o);
    hook_clients[key] = c;
    return c;
  }

  // Runs mutating webhooks; may modify `obj`. Throws StatusError on deny/failure.
  void call_webhooks(const TypeInfo& ti, const std::string& sub, const std::string& op, const std::string& ns,
                     const std::string& name, Value* obj, const Value* old, const UserInfo& user) {
    auto hooks = matching_webhooks(ti, sub, op);
    if (hooks.empty()) return;
    static auto& hist = metrics::Registry::global().histogram("kl_webhook_duration_seconds", "Webhook callout latency");
    static auto& calls = metrics::Registry::global().counter("kl_webhook_calls_total", "Webhook callouts (any outcome)");
    static auto& ring = [] () -> metrics::SampleLog& {
      auto& r = metrics::Registry::global().samples("webhook");
      r.link("kl_webhook_calls_total", &calls);  // counted with the sample, under its lock
      return r;
    }();
    for (const auto& hm : hooks) {
      const Value& hook = *hm.hook;
      std::string fail_policy = hook.get_string("failurePolicy", "Fail");
      int timeout_s = hook.get("timeoutSeconds").is_int() ? static_cast<int>(hook.get("timeoutSeconds").as_int()) : 10;
      std::string uid = crypto::uuid_v4();
      // AdmissionReview serialized in place: object/oldObject are dumped straight from the
      // caller's trees instead of being deep-copied into a request Value first.
      const std::string opts_kind = op == "CREATE" ? "CreateOptions" : op == "DELETE" ? "DeleteOptions" : "UpdateOptions";
      const std::string gvk = "{\"group\":" + json::quote(ti.rt.group) + ",\"version\":" + json::quote(ti.rt.version) +
                              ",\"kind\":" + json::quote(ti.rt.kind) + "}";
      const std::string gvr = "{\"group\":" + json::quote(ti.rt.group) + ",\"version\":" + json::quote(ti.rt.version) +
                              ",\"resource\":" + json::quote(ti.rt.plural) + "}";
      std::string body;
      body.reserve(1024 + (obj ? 2048 : 0) + (old ? 2048 : 0));
      body += "{\"kind\":\"AdmissionReview\",\"apiVersion\":\"admission.k8s.io/v1\",\"request\":{\"uid\":";
      body += json::quote(uid);
      body += ",\"kind\":" + gvk + ",\"resource\":" + gvr;
      if (!sub.empty()) body += ",\"subResource\":" + json::quote(sub);
      body += ",\"requestKind\":" + gvk + ",\"requestResource\":" + gvr;
      if (!sub.empty()) body += ",\"requestSubResource\":" + json::quote(sub);
      body += ",\"name\":" + json::quote(name);
      if (!ns.empty()) body += ",\"namespace\":" + json::quote(ns);
      body += ",\"operation\":" + json::quote(op);
      body += ",\"userInfo\":";
      user.to_json().dump_to(body);
      body += ",\"object\":";
      if (obj) obj->dump_to(body);
      else body += "null";
      body += ",\"oldObject\":";
      if (old) old->dump_to(body);
      else body += "null";
      body += ",\"dryRun\":false,\"options\":{\"kind\":" + json::quote(opts_kind) +
              ",\"apiVersion\":\"meta.k8s.io/v1\"}}}";
      std::string err;
      Value resp_review;
      int64_t t0 = metrics::now_ns();
      try {
        std::string path;
        auto client = hook_client(hm, path);
        http::Headers h;
        h.set("Content-Type", "application/json");
        h.set("Accept", "application/json");
        http::Response r = client->request("POST", path + "?timeout=" + std::to_string(timeout_s) + "s",
                                           body, &h, timeout_s * 1000);
        if (r.status != 200) {
          err = "expected webhook response status code 200, got " + std::to_string(r.status) + ": " + r.body;
        } else if (!json::try_parse(r.body, resp_review, &err)) {
          err = "failed to parse webhook response: " + err;
        }
      } catch (const std::exception& e) {
        err = e.what();
      }
      double secs = static_cast<double>(metrics::now_ns() - t0) * 1e-9;
      hist.observe(secs);
      ring.add(secs, &calls);
      const Value& resp = resp_review.get("response");
      if (err.empty() && !resp.is_object()) err = "webhook response was absent";
      if (err.empty() && resp.get_string("uid") != uid) {
        err = "expected response.uid=\"" + uid + "\", got \"" + resp.get_string("uid") + "\"";
      }
      if (!err.empty()) {
        if (fail_policy == "Ignore") {
          LOG_WARN("apiserver") << "failed calling webhook " << hm.name << " (ignored): " << err;
          continue;
        }
        throw StatusError(500, "InternalError",
                          "Internal error occurred: failed calling webhook \"" + hm.name + "\": " + err);
      }
      if (!resp.get("allowed").is_bool() || !resp.get("allowed").as_bool()) {
        const Value& st = resp.get("status");
        int code = st.get("code").is_int() ? static_cast<int>(st.get("code").as_int()) : 0;
        if (code < 400) code = 400;
        std::string reason = st.get_string("reason", code == 403 ? "Forbidden" : "BadRequest");
        std::string msg = "admission webhook \"" + hm.name + "\" denied the request";
        std::string m = st.get_string("message");
        msg += m.empty() ? " without explanation" : ": " + m;
        throw StatusError(code, reason, msg);
      }
      if (resp.get("patch").is_string() && obj) {
        if (resp.get_string("patchType", "JSONPatch") != "JSONPatch") {
          throw StatusError(500, "InternalError", "unsupported patchType from webhook " + hm.name);
        }
        Value patch;
        std::string perr;
        if (!json::try_parse(crypto::base64_decode(resp.get_string("patch")), patch, &perr)) {
          throw StatusError(500, "InternalError", "invalid patch from webhook " + hm.name + ": " + perr);
        }
        try {
          json::apply_patch(*obj, patch);
        } catch (const std::exception& e) {
          throw StatusError(500, "InternalError",
                            "Internal error occurred: failed calling webhook \"" + hm.name + "\": " + e.what());
        }
      }
    }
  }

  // ---------------------------------------------------------------- validation
  void validate_object(const TypeInfo& ti, const std::string& name, const std::string& ns, const Value& obj) {
    const Value& meta = obj.get("metadata");
    if (ti.rt.plural == "namespaces") {
      if (!dns1123_label(name)) {
        throw invalid(ti.rt, name, "metadata.name: Invalid value: \"" + name +
                                       "\": a lowercase RFC 1123 label must consist of lower case alphanumeric characters or '-', and must start and end with an alphanumeric character");
      }
    } else if (!dns1123_subdomain(name)) {
      throw invalid(ti.rt, name, "metadata.name: Invalid value: \"" + name +
                                     "\": a lowercase RFC 1123 subdomain must consist of lower case alphanumeric characters, '-' or '.', and must start and end with an alphanumeric character");
    }
    if (meta.get("namespace").is_string() && ti.rt.namespaced && meta.get_string("namespace") != ns) {
      throw StatusError(400, "BadRequest", "the namespace of the provided object does not match the namespace sent on the request");
    }
    for (const auto& ref : meta.get("ownerReferences").items()) {
      for (const char* f : {"apiVersion", "kind", "name", "uid"}) {
        if (!ref.get(f).is_string() || ref.get_string(f).empty()) {
          throw invalid(ti.rt, name, std::string("metadata.ownerReferences.") + f + ": Invalid value: \"\": " + f +
                                         " must not be empty");
        }
      }
    }
    if (ti.rt.plural == "rolebindings" || ti.rt.plural == "clusterrolebindings") {
      if (!obj.get("roleRef").is_object()) throw invalid(ti.rt, name, "roleRef: Required value");
    }
    std::shared_ptr<const Value> schema = std::atomic_load(&ti.schema);
    if (opts.validate_schema && ti.custom && schema && schema->is_object()) {
      auto errs = crd::validate(obj, *schema);
      if (!errs.empty()) {
        std::string msg;
        for (size_t i = 0; i < errs.size() && i < 5; ++i) {
          if (i) msg += ", ";
          const auto& e = errs[i];
          if (e.kind == "required") msg += e.path + ": Required value";
          else msg += e.path + ": Invalid value: " + e.detail;
        }
        throw invalid(ti.rt, name, msg);
      }
    }
  }

  // ---------------------------------------------------------------- CRDs
  // Called while holding the CRD type's exclusive lock; takes types_mu (lock order above).
  void register_crd(const Value& crd) {
    const Value& spec = crd.get("spec");
    std::string group = spec.get_string("group");
    const Value& names = spec.get("names");
    bool namespaced = spec.get_string("scope") == "Namespaced";
    StoreLock lk(types_mu, types_stats);
    for (const auto& v : spec.get("versions").items()) {
      if (v.get("served").is_bool() && !v.get("served").as_bool()) continue;
      TypeInfo ti;
      ti.rt.group = group;
      ti.rt.version = v.get_string("name");
      ti.rt.kind = names.get_string("kind");
      ti.rt.plural = names.get_string("plural");
      ti.rt.namespaced = namespaced;
      ti.rt.has_status = v.get("subresources").get("status").is_object();
      auto schema = std::make_shared<const Value>(v.get("schema").get("openAPIV3Schema"));
      ti.custom = true;
      auto it = types.find(ti.key());
      if (it != types.end()) {
        std::atomic_store(&it->second.schema, schema);  // CRD update: keep the storage, swap the schema
        continue;
      }
      ti.schema = schema;
      ti.store = std::make_shared<TypeStore>(opts.store_shards);
      types[ti.key()] = ti;
    }
  }

  // ---------------------------------------------------------------- storage helpers
  enum class NsPhase { Missing, Active, Terminating };
  NsPhase namespace_phase(const std::string& ns) {
    TypeInfo* nti = type_by_key(kube::types::Namespace.group + "/v1/namespaces");
    if (!nti) return NsPhase::Missing;
    const std::string key = obj_key(nti->rt, "", ns);
    auto& sh = nti->store->shard(key);
    SharedStoreLock lk(sh.mu, nti->store->stats);
    auto it = sh.objs.find(key);
    if (it == sh.objs.end()) return NsPhase::Missing;
    if (!it->second.obj->get("metadata").contains("deletionTimestamp")) return NsPhase::Active;
    return opts.namespace_termination ? NsPhase::Terminating : NsPhase::Missing;
  }

  static bool is_core_namespaces(const TypeInfo& ti) { return ti.rt.plural == "namespaces" && ti.rt.group.empty(); }

  // The namespace controller's deletion (k8s.io/kubernetes pkg/controller/namespace): mark
  // the namespace Terminating and queue its contents; the garbage collector deletes them and
  // then the namespace (its "kubernetes" spec finalizer).  Caller holds the shard lock.
  std::shared_ptr<const Value> terminate_namespace_locked(const TypeInfo& ti, const std::string& name, Stored& cur) {
    Value obj = *cur.obj;
    obj["metadata"]["deletionTimestamp"] = now_rfc3339();
    obj["metadata"]["deletionGracePeriodSeconds"] = 0;
    obj["status"]["phase"] = "Terminating";
    auto ptr = commit_locked(ti, "", name, std::move(obj), *cur.managers, &cur);
    std::lock_guard<std::mutex> g(gc_mu);
    gc_queue.push_back({true, name, true});
    gc_cv.notify_one();
    return ptr;
  }

  // Last step of a namespace's termination: its contents are gone; drop the spec finalizer
  // and remove it (unless metadata finalizers still hold it).
  void finish_namespace(const std::string& name) {
    TypeInfo* nti = type_by_key(kube::types::Namespace.group + "/v1/namespaces");
    if (!nti) return;
    const std::string key = obj_key(nti->rt, "", name);
    auto& sh = nti->store->shard(key);
    StoreLock lk(sh.mu, nti->store->stats);
    auto it = sh.objs.find(key);
    if (it == sh.objs.end() || !it->second.obj->get("metadata").contains("deletionTimestamp")) return;
    if (it->second.obj->get("metadata").get("finalizers").empty()) {
      erase_locked(*nti, "", name);
      return;
    }
    Value obj = *it->second.obj;
    if (obj.get("spec").get("finalizers").empty()) return;
    obj["spec"]["finalizers"] = Value::array();
    commit_locked(*nti, "", name, std::move(obj), *it->second.managers, &it->second);
  }

  static void render_managed(Value& obj, const Managers& m, const std::string& api_version) {
    Value arr = Value::array();
    for (const auto& [key, e] : m) {
      if (e.fields.empty()) continue;
      std::string mgr = key.substr(0, key.find('\x1f'));
      Value ent = Value::object({{"manager", mgr}, {"operation", e.operation},
                                 {"apiVersion", e.api_version.empty() ? api_version : e.api_version},
                                 {"time", e.time}, {"fieldsType", "FieldsV1"}, {"fieldsV1", fields_v1(e.fields)}});
      if (!e.subresource.empty()) ent["subresource"] = e.subresource;
      arr.push_back(std::move(ent));
    }
    if (arr.empty()) obj["metadata"].erase("managedFields");
    else obj["metadata"]["managedFields"] = std::move(arr);
  }

  // a == b ignoring metadata.managedFields and metadata.resourceVersion (no copies).
  static bool same_content(const Value& a, const Value& b) {
    if (!a.is_object() || !b.is_object()) return a == b;
    auto volatile_key = [](const std::string& k) { return k == "managedFields" || k == "resourceVersion"; };
    auto count = [&](const Value& v, bool meta) {
      size_t n = 0;
      for (const auto& k : v.keys()) n += (meta && volatile_key(k)) ? 0 : 1;
      return n;
    };
    if (a.size() != b.size()) return false;
    for (size_t i = 0; i < a.keys().size(); ++i) {
      const std::string& k = a.keys()[i];
      const Value* bv = b.find(k);
      if (!bv) return false;
      const Value& av = a.values()[i];
      if (k != "metadata") {
        if (!(av == *bv)) return false;
        continue;
      }
      if (!av.is_object() || !bv->is_object()) {
        if (!(av == *bv)) return false;
        continue;
      }
      if (count(av, true) != count(*bv, true)) return false;
      for (size_t j = 0; j < av.keys().size(); ++j) {
        const std::string& mk = av.keys()[j];
        if (volatile_key(mk)) continue;
        const Value* bm = bv->find(mk);
        if (!bm || !(av.values()[j] == *bm)) return false;
      }
    }
    return true;
  }

  // a != b outside metadata and status (no copies).
  static bool spec_changed(const Value& a, const Value& b) {
    if (!a.is_object() || !b.is_object()) return !(a == b);
    auto skip = [](const std::string& k) { return k == "metadata" || k == "status"; };
    size_t na = 0, nb = 0;
    for (size_t i = 0; i < a.keys().size(); ++i) {
      const std::string& k = a.keys()[i];
      if (skip(k)) continue;
      ++na;
      const Value* bv = b.find(k);
      if (!bv || !(a.values()[i] == *bv)) return true;
    }
    for (const auto& k : b.keys()) nb += skip(k) ? 0 : 1;
    return na != nb;
  }

  // Assign fields changed by a non-apply write to `manager`.
  static void attribute_update(Managers& m, const std::string& manager, const Value& before, const Value& after,
                               bool status_write, const std::string& api_version) {
    FieldSet changed, removed;
    // a status write replaces status alone (do_update / do_patch copy everything else
    // from the stored object), so only that subtree is diffed
    if (status_write) diff_member_leaves(before, after, "status", changed, removed);
    else diff_leaves(before, after, changed, removed);
    for (auto& [name, e] : m) {
      for (const auto& p : changed) e.fields.erase(p);
      for (const auto& p : removed) e.fields.erase(p);
    }
    if (!changed.empty()) {
      // managedFields entries are per (manager, subresource)
      auto& e = m[status_write ? manager + "\x1fstatus" : manager];
      if (e.operation.empty()) {
        e.operation = "Update";
        e.api_version = api_version;
      }
      if (e.operation == "Apply") {
        // an Update by an apply manager is tracked separately in k8s; keep it simple
        e.operation = "Update";
      }
      e.time = now_rfc3339();
      if (status_write) e.subresource = "status";
      for (const auto& p : changed) e.fields.insert(p);
    }
    for (auto it = m.begin(); it != m.end();) {
      if (it->second.fields.empty()) it = m.erase(it);
      else ++it;
    }
  }

  // Work moved out of the exclusive section: managedFields are rendered and the watch event
  // is serialized around a resourceVersion placeholder; commit_locked splices in the digits.
  static const std::string& rv_placeholder() {
    static const std::string p = "\x01rv\x01";
    return p;
  }
  static PreparedEvent prepare_commit(Value& obj, const Managers& managers, const std::string& api_version,
                                      const char* type) {
    obj["metadata"]["resourceVersion"] = rv_placeholder();
    render_managed(obj, managers, api_version);
    std::string line = std::string("{\"type\":\"") + type + "\",\"object\":";
    obj.dump_to(line);
    line += "}\n";
    static const std::string needle = "\"resourceVersion\":" + Value(rv_placeholder()).dump();
    PreparedEvent pe;
    pe.filter = filter_view(obj);
    pe.rec = std::make_shared<EventRec>();
    size_t pos = line.find(needle);
    if (pos == std::string::npos) return pe;
    pe.head.assign(line, 0, pos);
    pe.head += "\"resourceVersion\":\"";
    pe.tail.assign(line, pos + needle.size() - 1, std::string::npos);  // from the closing quote
    pe.ok = true;
    return pe;
  }

  // Commits `obj` (already validated).  Caller holds the object's shard exclusively; the
  // type's seq lock is taken here only to assign the resourceVersion and emit the event.
  // Returns the stored object; *dangling is set when every owner reference points at a
  // deleted object.
  std::shared_ptr<const Value> commit_locked(const TypeInfo& ti, const std::string& ns, const std::string& name,
                                            Value obj, Managers managers, const Stored* prev,
                                            const PreparedEvent* pe = nullptr, bool* dangling = nullptr,
                                            std::shared_ptr<const std::string>* line_out = nullptr) {
    TypeStore& ts = *ti.store;
    PreparedEvent local;
    if (!pe || !pe->ok) {
      local = prepare_commit(obj, managers, ti.rt.api_version(), prev ? "MODIFIED" : "ADDED");
      pe = &local;
    }
    std::string key = obj_key(ti.rt, ns, name);
    Ref ref{ti.key(), key};
    {
      // Indexed before the event is out: a client that reacts to it (creating a dependent
      // of this object) must find the owner in by_uid.  Indexed and checked in one critical
      // section: either the owner's deletion sees this dependent in by_owner (and the GC
      // removes it) or this check sees the owner gone.
      std::lock_guard<std::mutex> ig(index_mu);
      if (prev) unindex_owners_locked(*prev->obj, ref);
      by_uid[obj.get("metadata").get_string("uid")] = ref;
      const Value& owners = obj.get("metadata").get("ownerReferences");
      for (const auto& r : owners.items()) by_owner[r.get_string("uid")].insert(ref);
      if (ti.rt.namespaced) by_namespace[ns].insert(ref);
      if (dangling && !prev && !owners.empty()) {
        bool alive = false;
        for (const auto& r : owners.items()) alive = alive || by_uid.count(r.get_string("uid")) > 0;
        *dangling = !alive;
      }
    }
    // An update that changes the labels may move the object into or out of a label-selector
    // watch: the event remembers the previous version for those watches (view_for).
    std::shared_ptr<EventRec> rec = pe->rec ? pe->rec : std::make_shared<EventRec>();
    if (prev && opts.selector_transitions &&
        prev->obj->get("metadata").get("labels") != obj.get("metadata").get("labels")) {
      auto t = std::make_unique<EventRec::Transitions>();
      t->prev_meta = filter_view(*prev->obj);
      if (auto held = prev->line.lock()) {
        t->prev_line = std::move(held);
      } else {
        std::string l = "{\"type\":\"MODIFIED\",\"object\":";
        prev->obj->dump_to(l);
        l += "}\n";
        t->prev_line = std::make_shared<const std::string>(std::move(l));
      }
      rec->tr = std::move(t);
    }
    uint64_t new_rv;
    std::string digits;
    std::shared_ptr<const std::string> line;
    {
      StoreLock sl(ts.seq, ts.seq_stats);
      new_rv = ++rv;
      digits = rv_str(new_rv);
      std::string preline;
      if (pe->ok) {
        preline.reserve(pe->head.size() + digits.size() + pe->tail.size());
        preline += pe->head;
        preline += digits;
        preline += pe->tail;
      } else {  // no resourceVersion placeholder found (never for a prepared object)
        obj["metadata"]["resourceVersion"] = digits;
        preline = std::string("{\"type\":\"") + (prev ? "MODIFIED" : "ADDED") + "\",\"object\":";
        obj.dump_to(preline);
        preline += "}\n";
      }
      line = emit_locked(ti, ns, new_rv, std::move(preline), pe->filter ? pe->filter : filter_view(obj), std::move(rec));
    }
    obj["metadata"]["resourceVersion"] = digits;
    auto ptr = std::make_shared<const Value>(std::move(obj));
    Stored s;
    s.obj = ptr;
    s.rv = new_rv;
    s.managers = std::make_shared<const Managers>(std::move(managers));
    s.line = line;
    ts.shard(key).objs[key] = std::move(s);
    if (line_out) *line_out = std::move(line);
    return ptr;
  }

  void unindex_owners_locked(const Value& obj, const Ref& ref) {  // index_mu held
    for (const auto& r : obj.get("metadata").get("ownerReferences").items()) {
      auto it = by_owner.find(r.get_string("uid"));
      if (it == by_owner.end()) continue;
      it->second.erase(ref);
      if (it->second.empty()) by_owner.erase(it);
    }
  }

  // Removes an object and hands its dependents (and, for a Namespace, its contents) to the
  // garbage collector.  Caller holds the object's shard exclusively.
  void erase_locked(const TypeInfo& ti, const std::string& ns, const std::string& name) {
    TypeStore& ts = *ti.store;
    std::string key = obj_key(ti.rt, ns, name);
    auto& b = ts.shard(key).objs;
    auto it = b.find(key);
    if (it == b.end()) return;
    // The DELETED event carries the object at the new resourceVersion: its serialization is
    // split around the stored resourceVersion and the new digits are spliced in under seq.
    std::shared_ptr<const Value> ptr = it->second.obj;
    std::string line = "{\"type\":\"DELETED\",\"object\":";
    const size_t obj_at = line.size();
    static const std::string kObjectKey = ",\"object\":";
    const std::shared_ptr<const std::string> held = it->second.line.lock();
    const std::string* committed = held.get();
    const size_t at = committed ? committed->find(kObjectKey) : std::string::npos;
    if (at != std::string::npos && committed->size() >= at + kObjectKey.size() + 2) {
      // the object as its last commit serialized it (same tree, same rv digits)
      line.append(*committed, at + kObjectKey.size(), committed->size() - (at + kObjectKey.size()) - 2);
    } else {
      ptr->dump_to(line);
    }
    line += "}\n";
    const std::string old_rv = "\"resourceVersion\":" + json::quote(ptr->get("metadata").get_string("resourceVersion"));
    const size_t pos = line.find(old_rv, obj_at);
    auto filter = filter_view(*ptr);
    std::string uid = ptr->get("metadata").get_string("uid");
    Ref ref{ti.key(), key};
    bool has_dependents;
    {
      std::lock_guard<std::mutex> ig(index_mu);
      by_uid.erase(uid);
      unindex_owners_locked(*ptr, ref);
      if (ti.rt.namespaced) {
        auto nit = by_namespace.find(ns);
        if (nit != by_namespace.end()) {
          nit->second.erase(ref);
          if (nit->second.empty()) by_namespace.erase(nit);
        }
      }
      has_dependents = by_owner.count(uid) > 0;
    }
    uint64_t new_rv;
    {
      StoreLock sl(ts.seq, ts.seq_stats);
      new_rv = ++rv;
      const std::string digits = rv_str(new_rv);
      if (pos != std::string::npos) {
        line.replace(pos, old_rv.size(), "\"resourceVersion\":\"" + digits + "\"");
      } else {  // no resourceVersion in the stored object (never for committed objects)
        Value final_obj = *ptr;
        final_obj["metadata"]["resourceVersion"] = digits;
        line = "{\"type\":\"DELETED\",\"object\":";
        final_obj.dump_to(line);
        line += "}\n";
      }
      emit_locked(ti, ns, new_rv, std::move(line), std::move(filter), nullptr);
    }
    b.erase(it);
    bool is_ns = ti.rt.plural == "namespaces" && ti.rt.group.empty();
    if (has_dependents || is_ns) {
      std::lock_guard<std::mutex> g(gc_mu);
      if (has_dependents) gc_queue.push_back({false, uid});
      if (is_ns) gc_queue.push_back({true, name});
      gc_cv.notify_one();
    }
  }

  // Garbage collector thread: deletes dependents whose owners are all gone and the contents
  // of deleted namespaces, one type lock at a time.
  void gc_loop() {
    while (true) {
      GcItem item;
      {
        std::unique_lock<std::mutex> g(gc_mu);
        gc_cv.wait(g, [&] { return gc_stop || !gc_queue.empty(); });
        if (gc_stop) return;
        item = std::move(gc_queue.front());
        gc_queue.pop_front();
      }
      std::vector<Ref> victims;
      {
        std::lock_guard<std::mutex> ig(index_mu);
        auto& idx = item.is_namespace ? by_namespace : by_owner;
        auto it = idx.find(item.id);
        if (it != idx.end()) victims.assign(it->second.begin(), it->second.end());
      }
      for (const auto& v : victims) {
        TypeInfo* vti = type_by_key(v.first);
        if (!vti) continue;
        auto& vsh = vti->store->shard(v.second);
        StoreLock lk(vsh.mu, vti->store->stats);
        auto it = vsh.objs.find(v.second);
        if (it == vsh.objs.end()) continue;
        const Value& meta = it->second.obj->get("metadata");
        if (!item.is_namespace) {
          bool alive = false;
          {
            std::lock_guard<std::mutex> ig(index_mu);
            for (const auto& r : meta.get("ownerReferences").items()) alive = alive || by_uid.count(r.get_string("uid")) > 0;
          }
          if (alive) continue;
        }
        std::string vns = meta.get_string("namespace"), vname = meta.get_string("name");
        if (is_core_namespaces(*vti) && opts.namespace_termination) {
          if (!meta.contains("deletionTimestamp")) terminate_namespace_locked(*vti, vname, it->second);
          continue;
        }
        erase_locked(*vti, vns, vname);
        gc_collected.fetch_add(1, std::memory_order_relaxed);
      }
      if (item.finish_namespace) finish_namespace(item.id);
    }
  }

  // The apiserver decodes quantities into resource.Quantity and stores their canonical
  // form ("1000m" -> "1", "2048Mi" -> "2Gi"; a JSON number becomes a string).  kube-lite
  // does it for the quantity maps the product writes and reads back: ResourceQuota
  // spec.hard / status.hard / status.used and Node status.capacity / allocatable.
  static void canonicalize_quantities(const TypeInfo& ti, Value& obj) {
    if (ti.custom || (ti.rt.plural != "resourcequotas" && ti.rt.plural != "nodes")) return;
    auto fix = [](Value* m) {
      if (!m || !m->is_object()) return;
      for (Value& v : m->items_mut()) {
        std::string text;
        if (v.is_string()) text = v.as_string();
        else if (v.is_int()) text = v.dump();
        else continue;
        if (auto c = kube::canonical_quantity(text)) {
          if (!v.is_string() || *c != text) v = Value(std::move(*c));
        }
      }
    };
    auto sub = [](Value& o, const char* k) { return o.is_object() ? o.find_mut(k) : nullptr; };
    Value* spec = sub(obj, "spec");
    Value* status = sub(obj, "status");
    if (ti.rt.plural == "resourcequotas") {
      if (spec) fix(sub(*spec, "hard"));
      if (status) {
        fix(sub(*status, "hard"));
        fix(sub(*status, "used"));
      }
    } else if (status) {
      fix(sub(*status, "capacity"));
      fix(sub(*status, "allocatable"));
    }
  }

  // ---------------------------------------------------------------- write path
  using Compute = std::function<std::pair<Value, Managers>(const Stored* cur)>;

  // Generic optimistic write: compute (unlocked) -> admission (unlocked) -> validate ->
  // commit if the object did not change meanwhile (else retry).
  WriteResult write(TypeInfo& ti, const std::string& ns, const std::string& name, const std::string& sub,
                    const UserInfo& user, const Compute& compute, bool allow_create, bool is_status) {
    for (int attempt = 0; attempt < 8; ++attempt) {
      Stored cur_copy;
      bool exists = false;
      const std::string key = obj_key(ti.rt, ns, name);
      auto& sh = ti.store->shard(key);
      {
        SharedStoreLock lk(sh.mu, ti.store->stats);
        auto it = sh.objs.find(key);
        if (it != sh.objs.end()) {
          cur_copy = it->second;
          exists = true;
        }
      }
      if (!exists && !allow_create) throw not_found(ti.rt, name);
      auto [obj, managers] = compute(exists ? &cur_copy : nullptr);
      canonicalize_quantities(ti, obj);
      std::string op = exists ? "UPDATE" : "CREATE";
      if (!exists && ti.rt.namespaced) {
        const NsPhase phase = namespace_phase(ns);
        if (phase == NsPhase::Missing) {
          throw StatusError(404, "NotFound", "namespaces \"" + ns + "\" not found",
                            Value::object({{"name", ns}, {"kind", "namespaces"}}));
        }
        if (phase == NsPhase::Terminating) {
          throw StatusError(
              403, "Forbidden",
              ti.rt.plural + " \"" + name + "\" is forbidden: unable to create new content in namespace " + ns +
                  " because it is being terminated",
              Value::object({{"name", name}, {"kind", ti.rt.plural},
                             {"causes", Value::array({Value::object({{"reason", "NamespaceTerminating"},
                                                                     {"message", "namespace " + ns + " is being terminated"},
                                                                     {"field", "metadata.namespace"}})})}}));
        }
      }
      // no-op short-circuit (before admission, like the apiserver's update path)
      if (exists && same_content(obj, *cur_copy.obj) && managers == *cur_copy.managers) {
        return {cur_copy.obj, 200, nullptr};
      }
      trace_step(name, ".hook0");
      call_webhooks(ti, sub, op, ns, name, &obj, exists ? cur_copy.obj.get() : nullptr, user);
      trace_step(name, ".hook1");
      // identity fields cannot be changed by mutation
      obj["metadata"]["name"] = name;
      if (ti.rt.namespaced) obj["metadata"]["namespace"] = ns;
      else obj["metadata"].erase("namespace");
      canonicalize_quantities(ti, obj);  // a mutating webhook may have written quantities
      validate_object(ti, name, ns, obj);
      // everything below up to the lock depends only on cur_copy, which the commit re-checks
      if (exists && same_content(obj, *cur_copy.obj) && managers == *cur_copy.managers) {
        return {cur_copy.obj, 200, nullptr};  // mutation turned it into a no-op
      }
      if (exists && spec_changed(*cur_copy.obj, obj)) {
        int64_t gen = cur_copy.obj->get("metadata").get("generation").is_int()
                          ? cur_copy.obj->get("metadata").get("generation").as_int()
                          : 1;
        obj["metadata"]["generation"] = gen + 1;
      }
      PreparedEvent pe = prepare_commit(obj, managers, ti.rt.api_version(), exists ? "MODIFIED" : "ADDED");
      StoreLock lk(sh.mu, ti.store->stats);
      auto it = sh.objs.find(key);
      bool now_exists = it != sh.objs.end();
      if (now_exists != exists || (exists && it->second.rv != cur_copy.rv)) continue;  // raced: retry
      if (exists) {
        // finalizer-gated deletion completes when the last finalizer is removed
        // (a Terminating namespace waits for its contents: the spec finalizer)
        if (obj.get("metadata").contains("deletionTimestamp") && obj.get("metadata").get("finalizers").empty() &&
            !(is_core_namespaces(ti) && opts.namespace_termination && !obj.get("spec").get("finalizers").empty())) {
          erase_locked(ti, ns, name);
          return {cur_copy.obj, 200, nullptr};
        }
        (void)is_status;
        WriteResult wr;
        trace_step(name, ".commit");  // before the event is published: causally before its watch marks
        wr.obj = commit_locked(ti, ns, name, std::move(obj), std::move(managers), &it->second, &pe, nullptr, &wr.line);
        return wr;
      }
      if (ti.rt.plural == "customresourcedefinitions") register_crd(obj);
      bool dangling = false;
      std::shared_ptr<const std::string> line;
      trace_step(name, ".commit");
      auto created = commit_locked(ti, ns, name, std::move(obj), std::move(managers), nullptr, &pe, &dangling, &line);
      // The garbage collector also removes dependents created with only dangling owner
      // references (e.g. a controller re-applying a child right after its owner was
      // deleted, before the owner's DELETED event reached it).
      if (dangling) erase_locked(ti, ns, name);
      WriteResult wr;
      wr.obj = created;
      wr.code = 201;
      wr.line = std::move(line);
      return wr;
    }
    throw conflict(ti.rt, name);
  }

  // Fill server-populated metadata for a new object.
  void init_new(const TypeInfo& ti, Value& obj, const std::string& ns, const std::string& name) {
    obj["apiVersion"] = ti.rt.api_version();
    obj["kind"] = ti.rt.kind;
    Value& meta = obj["metadata"];
    meta["name"] = name;
    if (ti.rt.namespaced) meta["namespace"] = ns;
    meta["uid"] = crypto::uuid_v4();
    meta["creationTimestamp"] = now_rfc3339();
    meta["generation"] = 1;
    meta.erase("resourceVersion");
    meta.erase("deletionTimestamp");
    meta.erase("managedFields");
    if (ti.rt.has_status && ti.custom) obj.erase("status");
    if (ti.rt.plural == "namespaces" && ti.rt.group.empty()) {
      obj["spec"] = Value::object({{"finalizers", Value::array({"kubernetes"})}});
      obj["status"] = Value::object({{"phase", "Active"}});
    }
  }

  // Carry server-owned metadata from the stored object into an updated one.
  static void carry_meta(Value& obj, const Value& cur) {
    const Value& cm = cur.get("metadata");
    Value& m = obj["metadata"];
    for (const char* f : {"uid", "creationTimestamp", "generation", "deletionTimestamp"}) {
      if (cm.contains(f)) m[f] = cm.get(f);
      else m.erase(f);
    }
    obj["apiVersion"] = cur.get("apiVersion");
    obj["kind"] = cur.get("kind");
  }

  std::string field_manager(const http::Request& req, const std::string& dflt) {
    std::string fm = req.query_param("fieldManager");
    if (!fm.empty()) return fm;
    std::string ua = req.headers.get_or("User-Agent", dflt);
    size_t slash = ua.find('/');
    return slash == std::string::npos ? ua : ua.substr(0, slash);
  }

  Value parse_body(const http::Request& req) {
    Value v;
    std::string err;
    std::string ct = req.headers.get_or("Content-Type");
    if (ct.find("yaml") != std::string::npos && !req.body.empty() && req.body[0] != '{') {
      try {
        return yaml::parse(req.body);
      } catch (const std::exception& e) {
        throw StatusError(400, "BadRequest", std::string("error decoding YAML: ") + e.what());
      }
    }
    if (!json::try_parse(req.body, v, &err)) throw StatusError(400, "BadRequest", "couldn't get version/kind; json parse error: " + err);
    return v;
  }

  // ---------------------------------------------------------------- verbs
  void do_create(ParsedPath& p, const http::Request& req, const UserInfo& user, http::ResponseWriter& w) {
    Value body = parse_body(req);
    if (!body.is_object()) throw StatusError(400, "BadRequest", "object must be a JSON object");
    std::string name = body.get("metadata").get_string("name");
    if (name.empty()) {
      std::string gen = body.get("metadata").get_string("generateName");
      if (gen.empty()) throw invalid(p.ti->rt, "", "metadata.name: Required value: name or generateName is required");
      static const char* alnum = "bcdfghjklmnpqrstvwxz2456789";
      std::string rnd = crypto::random_bytes(5);
      name = gen;
      for (unsigned char c : rnd) name.push_back(alnum[c % 27]);
    }
    std::string manager = field_manager(req, "unknown");
    if (!t_trace_tag.empty()) t_trace_name = name;
    auto res = write(*p.ti, p.ns, name, "", user,
                     [&](const Stored* cur) -> std::pair<Value, Managers> {
                       if (cur) throw already_exists(p.ti->rt, name);
                       Value obj = body;
                       init_new(*p.ti, obj, p.ns, name);
                       Managers m;
                       attribute_update(m, manager, Value::object(), obj, false, p.ti->rt.api_version());
                       return {std::move(obj), std::move(m)};
                     },
                     true, false);
    {
      std::string_view b = res.body();
      if (!b.empty()) w.send_json(res.code, b);
      else w.send_json(res.code, res.obj->dump());
    }
  }

  void do_update(ParsedPath& p, const http::Request& req, const UserInfo& user, http::ResponseWriter& w) {
    Value body = parse_body(req);
    if (!body.is_object()) throw StatusError(400, "BadRequest", "object must be a JSON object");
    std::string bname = body.get("metadata").get_string("name");
    if (!bname.empty() && bname != p.name) {
      throw StatusError(400, "BadRequest", "the name of the object (" + bname +
                                               ") does not match the name on the URL (" + p.name + ")");
    }
    bool is_status = p.sub == "status";
    std::string manager = field_manager(req, "unknown");
    auto res = write(*p.ti, p.ns, p.name, p.sub, user,
                     [&](const Stored* cur) -> std::pair<Value, Managers> {
                       std::string want_rv = body.get("metadata").get_string("resourceVersion");
                       if (!want_rv.empty() && want_rv != cur->obj->get("metadata").get_string("resourceVersion")) {
                         throw conflict(p.ti->rt, p.name);
                       }
                       Value obj;
                       if (is_status) {
                         obj = *cur->obj;
                         if (body.contains("status")) obj["status"] = body.get("status");
                         else obj.erase("status");
                       } else {
                         obj = body;
                         carry_meta(obj, *cur->obj);
                         if (p.ti->rt.has_status) {
                           if (cur->obj->contains("status")) obj["status"] = cur->obj->get("status");
                           else obj.erase("status");
                         }
                       }
                       Managers m = *cur->managers;
                       attribute_update(m, manager, *cur->obj, obj, is_status, p.ti->rt.api_version());
                       return {std::move(obj), std::move(m)};
                     },
                     false, is_status);
    {
      std::string_view b = res.body();
      if (!b.empty()) w.send_json(res.code, b);
      else w.send_json(res.code, res.obj->dump());
    }
  }

  std::pair<Value, Managers> apply_ssa(const TypeInfo& ti, const Stored* cur, const Value& config,
                                       const std::string& manager_name, bool force, bool is_status,
                                       const std::string& ns, const std::string& name) {
    const std::string manager = is_status ? manager_name + "\x1fstatus" : manager_name;
    FieldSet cfg_fields = leaves(config, is_status);
    if (is_status) {
      FieldSet only;
      for (const auto& f : cfg_fields) {
        if (f == "/status" || f.rfind("/status/", 0) == 0) only.insert(f);
      }
      cfg_fields.swap(only);
    }
    Value live;
    Managers m;
    if (cur) {
      live = *cur->obj;
      m = *cur->managers;
    } else {
      live = Value::object();
      init_new(ti, live, ns, name);
    }
    // conflicts with other managers owning a field with a different value
    std::vector<std::pair<std::string, std::string>> conflicts;
    for (const auto& f : cfg_fields) {
      const Value* want = get_path(config, f);
      const Value* have = get_path(live, f);
      for (auto& [other, e] : m) {
        if (other == manager || !e.fields.count(f)) continue;
        if (have && want && *have == *want) continue;
        conflicts.emplace_back(other, f);
      }
    }
    if (!conflicts.empty() && !force) {
      std::string msg = "Apply failed with " + std::to_string(conflicts.size()) + " conflict" +
                        (conflicts.size() > 1 ? "s" : "") + ": ";
      for (size_t i = 0; i < conflicts.size(); ++i) {
        if (i) msg += "; ";
        msg += "conflict with \"" + conflicts[i].first.substr(0, conflicts[i].first.find('\x1f')) + "\": " +
               display_path(conflicts[i].second);
      }
      throw StatusError(409, "Conflict", msg);
    }
    if (force) {
      for (const auto& [other, f] : conflicts) m[other].fields.erase(f);
    }
    // prune fields this manager owned but no longer applies (and nobody else owns)
    if (auto it = m.find(manager); it != m.end()) {
      for (const auto& f : it->second.fields) {
        if (cfg_fields.count(f)) continue;
        bool other_owner = false;
        for (auto& [other, e] : m) {
          if (other != manager && e.fields.count(f)) other_owner = true;
        }
        if (!other_owner) remove_path(live, f);
      }
    }
    for (const auto& f : cfg_fields) {
      if (const Value* v = get_path(config, f)) set_path(live, f, *v);
    }
    // shared fields: other managers co-own identical values
    auto& me = m[manager];
    me.operation = "Apply";
    me.api_version = ti.rt.api_version();
    me.time = now_rfc3339();
    me.subresource = is_status ? "status" : "";
    me.fields = cfg_fields;
    for (auto it = m.begin(); it != m.end();) {
      if (it->second.fields.empty()) it = m.erase(it);
      else ++it;
    }
    if (cur && ti.rt.has_status && !is_status) {
      if (cur->obj->contains("status")) live["status"] = cur->obj->get("status");
    }
    return {std::move(live), std::move(m)};
  }

  void do_patch(ParsedPath& p, const http::Request& req, const UserInfo& user, http::ResponseWriter& w) {
    std::string ct = req.headers.get_or("Content-Type");
    bool is_status = p.sub == "status";
    bool is_apply = ct.find("apply-patch") != std::string::npos;
    std::string manager = field_manager(req, is_apply ? "" : "unknown");
    if (is_apply && req.query_param("fieldManager").empty()) {
      throw StatusError(400, "BadRequest", "PatchOptions.meta.k8s.io \"\" is invalid: fieldManager: Required value: is required for apply patch");
    }
    Value patch = parse_body(req);
    bool force = req.query_param("force") == "true";
    auto res = write(*p.ti, p.ns, p.name, p.sub, user,
                     [&](const Stored* cur) -> std::pair<Value, Managers> {
                       if (is_apply) {
                         std::string pname = patch.get("metadata").get_string("name");
                         if (!pname.empty() && pname != p.name) {
                           throw StatusError(400, "BadRequest", "the name of the object (" + pname +
                                                                    ") does not match the name on the URL (" + p.name + ")");
                         }
                         return apply_ssa(*p.ti, cur, patch, manager, force, is_status, p.ns, p.name);
                       }
                       Value obj = *cur->obj;
                       try {
                         if (ct.find("json-patch") != std::string::npos) {
                           json::apply_patch(obj, patch);
                         } else {
                           json::apply_merge_patch(obj, patch);
                         }
                       } catch (const json::PatchError& e) {
                         throw StatusError(422, "Invalid", std::string("the server rejected our request due to an error in our request: ") + e.what());
                       }
                       std::string want_rv = obj.get("metadata").get_string("resourceVersion");
                       if (!want_rv.empty() && want_rv != cur->obj->get("metadata").get_string("resourceVersion")) {
                         throw conflict(p.ti->rt, p.name);
                       }
                       if (is_status) {
                         Value keep = *cur->obj;
                         if (obj.contains("status")) keep["status"] = obj.get("status");
                         else keep.erase("status");
                         obj = std::move(keep);
                       } else {
                         carry_meta(obj, *cur->obj);
                         if (p.ti->rt.has_status) {
                           if (cur->obj->contains("status")) obj["status"] = cur->obj->get("status");
                           else obj.erase("status");
                         }
                       }
                       Managers m = *cur->managers;
                       attribute_update(m, manager, *cur->obj, obj, is_status, p.ti->rt.api_version());
                       return {std::move(obj), std::move(m)};
                     },
                     is_apply, is_status);
    {
      std::string_view b = res.body();
      if (!b.empty()) w.send_json(res.code, b);
      else w.send_json(res.code, res.obj->dump());
    }
  }

  void do_delete(ParsedPath& p, const http::Request& req, const UserInfo& user, http::ResponseWriter& w) {
    std::shared_ptr<const Value> cur;
    const std::string key = obj_key(p.ti->rt, p.ns, p.name);
    auto& sh = p.ti->store->shard(key);
    {
      SharedStoreLock lk(sh.mu, p.ti->store->stats);
      auto it = sh.objs.find(key);
      if (it == sh.objs.end()) throw not_found(p.ti->rt, p.name);
      cur = it->second.obj;
    }
    trace_step(p.name, ".hook0");
    call_webhooks(*p.ti, "", "DELETE", p.ns, p.name, nullptr, cur.get(), user);
    trace_step(p.name, ".hook1");
    StoreLock lk(sh.mu, p.ti->store->stats);
    auto it = sh.objs.find(key);
    if (it == sh.objs.end()) throw not_found(p.ti->rt, p.name);
    const Value& meta = it->second.obj->get("metadata");
    if (is_core_namespaces(*p.ti) && opts.namespace_termination) {
      auto ptr = meta.contains("deletionTimestamp") ? it->second.obj
                                                    : terminate_namespace_locked(*p.ti, p.name, it->second);
      w.send_json(200, ptr->dump());
      return;
    }
    if (!meta.get("finalizers").empty()) {
      if (!meta.contains("deletionTimestamp")) {
        Value obj = *it->second.obj;
        obj["metadata"]["deletionTimestamp"] = now_rfc3339();
        obj["metadata"]["deletionGracePeriodSeconds"] = 0;
        auto ptr = commit_locked(*p.ti, p.ns, p.name, std::move(obj), *it->second.managers, &it->second);
        w.send_json(202, ptr->dump());
        return;
      }
      w.send_json(202, it->second.obj->dump());
      return;
    }
    erase_locked(*p.ti, p.ns, p.name);
    (void)req;
    w.send_json(200, status_body(200, "", "").dump());
  }

  void do_get(ParsedPath& p, http::ResponseWriter& w, bool meta_only = false) {
    std::shared_ptr<const Value> obj;
    {
      const std::string key = obj_key(p.ti->rt, p.ns, p.name);
      auto& sh = p.ti->store->shard(key);
      SharedStoreLock lk(sh.mu, p.ti->store->stats);
      auto it = sh.objs.find(key);
      if (it == sh.objs.end()) throw not_found(p.ti->rt, p.name);
      obj = it->second.obj;
    }
    if (meta_only) {
      std::string out;
      dump_partial_metadata(*obj, out);
      w.send_json(200, out);
      return;
    }
    w.send_json(200, obj->dump());
  }

  void do_list(ParsedPath& p, const http::Request& req, http::ResponseWriter& w) {
    const int64_t limit = req.has_query_param("limit") ? std::atoll(req.query_param("limit").c_str()) : 0;
    const std::string cont = req.query_param("continue");
    std::vector<std::shared_ptr<const Value>> items;
    uint64_t list_rv = 0;
    size_t offset = 0;
    uint64_t snap_id = 0;
    if (!cont.empty()) {
      // "<snapshot id>.<offset>": later pages come from the first page's snapshot, so a
      // paginated LIST is consistent at one resourceVersion (as etcd serves it)
      const size_t dot = cont.find('.');
      snap_id = std::strtoull(cont.c_str(), nullptr, 10);
      offset = dot == std::string::npos ? 0 : std::strtoull(cont.c_str() + dot + 1, nullptr, 10);
      std::lock_guard<std::mutex> lk(list_mu);
      auto it = list_snapshots.find(snap_id);
      if (it == list_snapshots.end() || std::chrono::steady_clock::now() > it->second.expires) {
        if (it != list_snapshots.end()) list_snapshots.erase(it);
        throw StatusError(410, "Expired",
                          "The provided continue parameter is too old to display a consistent list result. You can "
                          "start a new list without the continue parameter.");
      }
      list_rv = it->second.rv;
      items = it->second.items;  // shared pointers only
    } else {
      auto sel = parse_selector(req.query_param("labelSelector"));
      auto ff = parse_field_selector(req.query_param("fieldSelector"));
      {
        // no commit of this type is in flight while we hold all its shards, so every event
        // of this type with rv <= list_rv is reflected in the items
        AllShards lk(*p.ti->store, false);
        list_rv = rv.load();
        for (auto& sh : p.ti->store->shards)
        for (auto& [k, st] : sh.objs) {
          const Value& meta = st.obj->get("metadata");
          if (!p.ns.empty() && meta.get_string("namespace") != p.ns) continue;
          if (!ff.name_ok(meta.get_string("name"))) continue;
          if (!ff.ns.empty() && meta.get_string("namespace") != ff.ns) continue;
          if (!sel.empty() && !selector_matches(sel, *st.obj)) continue;
          items.push_back(st.obj);
        }
      }
      std::sort(items.begin(), items.end(), [](const auto& a, const auto& b) {
        const Value& ma = a->get("metadata");
        const Value& mb = b->get("metadata");
        return std::make_pair(ma.get_string("namespace"), ma.get_string("name")) <
               std::make_pair(mb.get_string("namespace"), mb.get_string("name"));
      });
    }
    size_t end = items.size();
    std::string next;
    if (limit > 0 && offset + static_cast<size_t>(limit) < items.size()) {
      end = offset + static_cast<size_t>(limit);
      std::lock_guard<std::mutex> lk(list_mu);
      if (snap_id == 0) {
        const auto now = std::chrono::steady_clock::now();
        for (auto it = list_snapshots.begin(); it != list_snapshots.end();) {
          it = now > it->second.expires ? list_snapshots.erase(it) : std::next(it);
        }
        snap_id = next_list_id++;
        list_snapshots[snap_id] = ListSnapshot{list_rv, items, now + std::chrono::milliseconds(opts.continue_ttl_ms)};
      }
      next = std::to_string(snap_id) + "." + std::to_string(end);
    } else if (snap_id != 0) {
      std::lock_guard<std::mutex> lk(list_mu);
      list_snapshots.erase(snap_id);  // last page served
    }
    if (limit > 0) list_pages.fetch_add(1);
    const bool meta_only = wants_metadata(req);
    std::string out = meta_only ? std::string("{\"apiVersion\":\"meta.k8s.io/v1\",\"kind\":\"PartialObjectMetadataList\"")
                                : "{\"apiVersion\":" + json::quote(p.ti->rt.api_version()) + ",\"kind\":" +
                                      json::quote(p.ti->rt.kind + "List");
    out += ",\"metadata\":{\"resourceVersion\":\"" + rv_str(list_rv) + "\"";
    if (!next.empty()) {
      out += ",\"continue\":" + json::quote(next) +
             ",\"remainingItemCount\":" + std::to_string(items.size() - end);
    }
    out += "},\"items\":[";
    for (size_t i = offset; i < end; ++i) {
      if (i != offset) out.push_back(',');
      if (meta_only) dump_partial_metadata(*items[i], out);
      else items[i]->dump_to(out);
    }
    out += "]}";
    w.send_json(200, out);
  }

  void do_watch(ParsedPath& p, const http::Request& req, http::ResponseWriter& w) {
    auto subp = std::make_shared<WatchSub>();  // shared: a committer may still hold it for a wake-up
    WatchSub& sub = *subp;
    sub.type_key = p.ti->key();
    sub.ns = p.ns;
    sub.sel = parse_selector(req.query_param("labelSelector"));
    sub.fields = parse_field_selector(req.query_param("fieldSelector"));
    if (!sub.fields.ns.empty()) sub.ns = sub.fields.ns;
    std::string rv_s = req.query_param("resourceVersion");
    const bool meta_only = wants_metadata(req);
    int timeout_s = opts.max_watch_seconds;
    if (req.has_query_param("timeoutSeconds")) timeout_s = std::min(timeout_s, std::atoi(req.query_param("timeoutSeconds").c_str()));
    bool bookmarks = req.query_param("allowWatchBookmarks") == "true";
    const std::string trace_watch = "kl.watch." + p.ti->rt.plural + "." + field_manager(req, "unknown") + ".sent";
    const std::string trace_written = trace_watch.substr(0, trace_watch.size() - 4) + "written";
    const std::string slow_write = "kw:" + p.ti->rt.plural + " write";
    // the serving thread streams this watch from here on: name it for per-thread CPU reports
    set_thread_name("kw:" + p.ti->rt.plural);
    struct Rename {
      ~Rename() { set_thread_name("conn:apiserver"); }
    } rename;
    // Streaming lists (WatchList): sendInitialEvents=true replays the current state as
    // ADDED events, then a BOOKMARK annotated k8s.io/initial-events-end marks the point
    // where the initial state is complete (requires allowWatchBookmarks and
    // resourceVersionMatch=NotOlderThan, as on a real apiserver).
    const bool send_initial = req.query_param("sendInitialEvents") == "true";
    if (send_initial && (!bookmarks || req.query_param("resourceVersionMatch") != "NotOlderThan")) {
      throw StatusError(422, "Invalid",
                        "sendInitialEvents requires allowWatchBookmarks=true and resourceVersionMatch=NotOlderThan");
    }
    uint64_t from = 0;
    if (!rv_s.empty() && rv_s != "0" && !parse_rv(rv_s, &from)) {
      throw StatusError(400, "BadRequest", "invalid resource version: " + rv_s);
    }
    std::vector<std::shared_ptr<const std::string>> initial;
    bool gone = false;
    TypeStore& ts = *p.ti->store;
    uint64_t compacted = 0;
    uint64_t initial_rv = 0;
    {
      // No event of this type can interleave between the snapshot / history scan and the
      // registration below: a snapshot holds every shard (no commit of the type in flight),
      // a history replay holds seq (where commits append their events).
      const bool snapshot = rv_s.empty() || rv_s == "0" || send_initial;
      std::optional<AllShards> shards_lk;
      if (snapshot) shards_lk.emplace(ts, false);
      SharedStoreLock lk(ts.seq, ts.seq_stats);
      compacted = ts.compacted_rv;
      initial_rv = rv.load();
      if (snapshot) {
        for (auto& sh : ts.shards)
        for (auto& [k, st] : sh.objs) {
          const Value& meta = st.obj->get("metadata");
          if (!sub.ns.empty() && meta.get_string("namespace") != sub.ns) continue;
          if (!sub.fields.name_ok(meta.get_string("name"))) continue;
          if (!sub.sel.empty() && !selector_matches(sub.sel, *st.obj)) continue;
          std::string line = "{\"type\":\"ADDED\",\"object\":";
          if (meta_only) dump_partial_metadata(*st.obj, line);
          else st.obj->dump_to(line);
          line += "}\n";
          initial.push_back(std::make_shared<const std::string>(std::move(line)));
        }
      } else if (from < ts.compacted_rv) {
        gone = true;
      } else {
        auto it = std::upper_bound(ts.history.begin(), ts.history.end(), from,
                                   [](uint64_t v, const std::shared_ptr<const EventRec>& e) { return v < e->rv; });
        for (; it != ts.history.end(); ++it) {
          const auto& e = *it;
          if (e->type_key != sub.type_key) continue;
          if (!sub.ns.empty() && e->ns != sub.ns) continue;
          if (!sub.fields.name_ok(e->meta->get("metadata").get_string("name"))) continue;
          View view;
          if (!view_for(sub.sel, *e, &view)) continue;
          if (view == View::AsIs && !meta_only) initial.push_back(e->line);
          else initial.push_back(std::make_shared<const std::string>(e->line_as(view, meta_only)));
        }
      }
      if (!gone) {
        std::lock_guard<std::mutex> wg(ts.watches_mu);
        ts.watches.insert(subp);
      }
    }
    if (!w.start_chunked(200, "application/json")) {
      std::lock_guard<std::mutex> wg(ts.watches_mu);
      ts.watches.erase(subp);
      return;
    }
    if (gone) {
      Value ev = Value::object({{"type", "ERROR"},
                                {"object", status_body(410, "Expired", "too old resource version: " + rv_s + " (" +
                                                                           rv_str(compacted) + ")")}});
      w.write_chunk(ev.dump() + "\n");
      w.end_chunked();
      return;
    }
    bool ok = true;
    for (auto& l : initial) {
      if (!(ok = w.write_chunk(*l))) break;
    }
    if (ok && send_initial) {
      Value bm = Value::object(
          {{"type", "BOOKMARK"},
           {"object", Value::object({{"kind", p.ti->rt.kind},
                                     {"apiVersion", p.ti->rt.api_version()},
                                     {"metadata", Value::object({{"resourceVersion", rv_str(initial_rv)},
                                                                 {"annotations", Value::object({{"k8s.io/initial-events-end", "true"}})}})}})}});
      ok = w.write_chunk(bm.dump() + "\n");
    }
    auto deadline = std::chrono::steady_clock::now() + std::chrono::seconds(timeout_s);
    auto next_bookmark = std::chrono::steady_clock::now() + std::chrono::milliseconds(opts.bookmark_interval_ms);
    while (ok && !w.stopping()) {
      std::vector<QueuedEvent> batch;
      bool closed = false, overflow = false;
      {
        std::unique_lock<std::mutex> lk(sub.m);
        sub.cv.wait_for(lk, std::chrono::milliseconds(500), [&] { return !sub.q.empty() || sub.closed || sub.overflow; });
        const int coalesce_us = watch_coalesce_us.load(std::memory_order_relaxed);
        if (coalesce_us > 0 && !sub.q.empty() && sub.q.size() < 16 && !sub.closed) {
          // let a burst accumulate into one write (see Options::watch_coalesce_us)
          sub.cv.wait_for(lk, std::chrono::microseconds(coalesce_us),
                          [&] { return sub.q.size() >= 16 || sub.closed || sub.overflow; });
        }
        batch.assign(sub.q.begin(), sub.q.end());
        sub.q.clear();
        closed = sub.closed;
        overflow = sub.overflow;
      }
      if (!batch.empty()) {
        std::string buf;
        for (auto& q : batch) buf += q.e->line_as(q.view, meta_only);
        const bool traced = trace::armed();
        if (traced) {  // before the write: causally before the watcher's own marks
          for (auto& q : batch) trace::mark(q.e->meta->get("metadata").get_string("name"), trace_watch);
        }
        const int64_t w0 = metrics::now_ns();
        if (!w.write_chunk(buf)) break;
        const int64_t w1 = metrics::now_ns();
        stall::note_slow(slow_write, w0, w1);
        if (traced) {
          for (auto& q : batch) trace::mark_at(q.e->meta->get("metadata").get_string("name"), trace_written, w1);
        }
      }
      if (closed || overflow) break;
      auto now = std::chrono::steady_clock::now();
      if (now >= deadline) break;
      if (bookmarks && now >= next_bookmark) {
        // Under the type's shared lock every event of this type with rv <= cur_rv is already
        // in sub.q; flush those before the bookmark so it never skips an undelivered event.
        uint64_t cur_rv;
        std::vector<QueuedEvent> pending;
        {
          SharedStoreLock lk(ts.seq, ts.seq_stats);  // every event of the type up to cur_rv is queued
          cur_rv = rv.load();
          std::lock_guard<std::mutex> g(sub.m);
          pending.assign(sub.q.begin(), sub.q.end());
          sub.q.clear();
        }
        if (!pending.empty()) {
          std::string buf;
          for (auto& q : pending) buf += q.e->line_as(q.view, meta_only);
          if (!w.write_chunk(buf)) break;
        }
        Value bm = Value::object({{"type", "BOOKMARK"},
                                  {"object", Value::object({{"kind", p.ti->rt.kind},
                                                            {"apiVersion", p.ti->rt.api_version()},
                                                            {"metadata", Value::object({{"resourceVersion", rv_str(cur_rv)}})}})}});
        if (!w.write_chunk(bm.dump() + "\n")) break;
        next_bookmark = now + std::chrono::milliseconds(opts.bookmark_interval_ms);
      }
      if (batch.empty() && w.peer_closed()) break;
    }
    {
      std::lock_guard<std::mutex> wg(ts.watches_mu);
      ts.watches.erase(subp);
    }
    w.end_chunked();
  }

  // ---------------------------------------------------------------- discovery
  void discovery(const std::string& path, http::ResponseWriter& w) {
    SharedStoreLock lk(types_mu, types_stats);
    if (path == "/api") {
      w.send_json(200, Value::object({{"kind", "APIVersions"}, {"versions", Value::array({"v1"})}}).dump());
      return;
    }
    if (path == "/apis") {
      std::map<std::string, std::set<std::string>> groups;
      for (auto& [k, ti] : types) {
        if (!ti.rt.group.empty()) groups[ti.rt.group].insert(ti.rt.version);
      }
      Value gl = Value::array();
      for (auto& [g, vs] : groups) {
        Value versions = Value::array();
        for (auto& v : vs) versions.push_back(Value::object({{"groupVersion", g + "/" + v}, {"version", v}}));
        gl.push_back(Value::object({{"name", g}, {"versions", versions}, {"preferredVersion", versions[0]}}));
      }
      w.send_json(200, Value::object({{"kind", "APIGroupList"}, {"apiVersion", "v1"}, {"groups", gl}}).dump());
      return;
    }
    std::string gv = path.rfind("/api/", 0) == 0 ? path.substr(5) : path.substr(6);
    Value res = Value::array();
    for (auto& [k, ti] : types) {
      if (ti.rt.api_version() != gv) continue;
      Value verbs = Value::array({"create", "delete", "get", "list", "patch", "update", "watch"});
      res.push_back(Value::object({{"name", ti.rt.plural}, {"namespaced", ti.rt.namespaced}, {"kind", ti.rt.kind}, {"verbs", verbs}}));
      if (ti.rt.has_status) {
        res.push_back(Value::object({{"name", ti.rt.plural + "/status"}, {"namespaced", ti.rt.namespaced}, {"kind", ti.rt.kind},
                                     {"verbs", Value::array({"get", "patch", "update"})}}));
      }
    }
    if (res.empty()) throw StatusError(404, "NotFound", "the server could not find the requested resource");
    w.send_json(200, Value::object({{"kind", "APIResourceList"}, {"apiVersion", "v1"}, {"groupVersion", gv}, {"resources", res}}).dump());
  }

  // ---------------------------------------------------------------- faults
  // Fault injection's response hold (FaultRule::hold_ms): every writer call is forwarded to
  // the connection's writer, send() after waiting out the hold.  Not used for watches.
  class HoldingWriter : public http::ResponseWriter {
   public:
    HoldingWriter(http::ResponseWriter& inner, int hold_ms)
        : ResponseWriter(nullptr, inner.keep_alive(), never_stops()), inner_(inner), hold_ms_(hold_ms) {}
    void send(int status, std::string_view body, const std::string& content_type,
              const http::Headers* extra) override {
      inner_.wait_stopping(std::chrono::milliseconds(hold_ms_));
      inner_.send(status, body, content_type, extra);
      sent_ = true;
      status_ = status;
    }
    bool start_chunked(int status, const std::string& content_type) override {
      sent_ = true;
      status_ = status;
      return inner_.start_chunked(status, content_type);
    }
    bool write_chunk(const std::string& data) override { return inner_.write_chunk(data); }
    void end_chunked() override { inner_.end_chunked(); }
    void abort() override { inner_.abort(); }
    bool peer_closed() override { return inner_.peer_closed(); }
    const char* protocol() const override { return inner_.protocol(); }

   private:
    static const CancelToken& never_stops() {
      static const CancelToken t;
      return t;
    }
    http::ResponseWriter& inner_;
    int hold_ms_;
  };

  bool inject_fault(const http::Request& req, http::ResponseWriter& w, int* hold_ms) {
    FaultRule hit;
    bool found = false;
    {
      std::lock_guard<std::mutex> lk(fault_mu);
      for (auto& f : faults) {
        if (f.remaining == 0) continue;
        if (!f.method.empty() && f.method != req.method) continue;
        std::string target = req.path + (req.query.empty() ? "" : "?" + req.query);
        if (!std::regex_search(target, f.path)) continue;
        if (f.remaining > 0) --f.remaining;
        hit = f;
        found = true;
        break;
      }
    }
    if (!found) return false;
    faults_hit.fetch_add(1);
    // a delay ends early when the server stops, so no handler outlives it
    if (hit.delay_ms > 0 && w.wait_stopping(std::chrono::milliseconds(hit.delay_ms))) {
      w.abort();
      return true;
    }
    if (hit.reset) {
      w.abort();
      return true;
    }
    if (hit.hold_ms > 0 && hit.status <= 0) {
      *hold_ms = hit.hold_ms;
      return false;
    }
    if (hit.status > 0) {
      std::string reason = hit.status == 409   ? "Conflict"
                           : hit.status == 410 ? "Expired"
                           : hit.status == 429 ? "TooManyRequests"
                           : hit.status >= 500 ? "InternalError"
                                               : "BadRequest";
      http::Headers extra;
      if (hit.retry_after_s >= 0) extra.set("Retry-After", std::to_string(hit.retry_after_s));
      w.send(hit.status, status_body(hit.status, reason, hit.message.empty() ? "injected fault" : hit.message).dump(),
             "application/json", &extra);
      return true;
    }
    return false;
  }

  void control(http::Request& req, http::ResponseWriter& w) {
    if (req.path == "/_kl/faults" && req.method == "POST") {
      Value rules = json::parse(req.body);
      std::lock_guard<std::mutex> lk(fault_mu);
      if (req.query_param("append") != "true") faults.clear();
      for (const auto& r : rules.items()) {
        FaultRule f;
        f.method = r.get_string("method");
        f.path_src = r.get_string("path", ".*");
        f.path = std::regex(f.path_src);
        f.status = r.get("status").is_int() ? static_cast<int>(r.get("status").as_int()) : 0;
        f.delay_ms = r.get("delay_ms").is_int() ? static_cast<int>(r.get("delay_ms").as_int()) : 0;
        f.hold_ms = r.get("delay_response_ms").is_int() ? static_cast<int>(r.get("delay_response_ms").as_int()) : 0;
        f.remaining = r.get("count").is_int() ? static_cast<int>(r.get("count").as_int()) : -1;
        f.message = r.get_string("message");
        f.reset = r.get("reset").is_bool() && r.get("reset").as_bool();
        f.retry_after_s = r.get("retry_after").is_int() ? static_cast<int>(r.get("retry_after").as_int()) : -1;
        faults.push_back(std::move(f));
      }
      w.send_json(200, "{}");
      return;
    }
    if (req.path == "/_kl/faults" && req.method == "DELETE") {
      std::lock_guard<std::mutex> lk(fault_mu);
      faults.clear();
      w.send_json(200, "{}");
      return;
    }
    if (req.path == "/_kl/write-latency-us" && req.method == "POST") {
      // body: microseconds of storage commit latency for later writes
      try {
        size_t used = 0;
        const long long us = std::stoll(req.body, &used);
        if (us < 0 || us > 10000000) throw std::out_of_range("write latency");
        write_latency_us = us;
      } catch (const std::exception&) {
        w.send(400, "body must be 0..10000000 microseconds\n");
        return;
      }
      w.send(200, std::to_string(write_latency_us.load()) + "\n");
      return;
    }
    if (req.path == "/_kl/watch-coalesce-us" && req.method == "POST") {
      // body: microseconds a watch writer waits for a burst to grow before writing (0 = off);
      // answers the previous value, so a caller can restore it
      int prev = 0;
      try {
        size_t used = 0;
        const long us = std::stol(req.body, &used);
        if (us < 0 || us > 100000) throw std::out_of_range("watch coalesce");
        prev = watch_coalesce_us.exchange(static_cast<int>(us));
      } catch (const std::exception&) {
        w.send(400, "body must be 0..100000 microseconds\n");
        return;
      }
      w.send(200, std::to_string(prev) + "\n");
      return;
    }
    if (req.path == "/_kl/webhook-protocol" && req.method == "POST") {
      // body "h2" or "http/1.1": later webhook calls use fresh clients of that protocol
      const bool h2 = req.body == "h2";
      if (!h2 && req.body != "http/1.1") {
        w.send(400, "body must be h2 or http/1.1\n");
        return;
      }
      {
        std::lock_guard<std::mutex> lk(hook_mu);
        webhook_h2 = h2;
        hook_fast.clear();
        hook_clients.clear();
      }
      w.send(200, h2 ? "h2\n" : "http/1.1\n");
      return;
    }
    if (req.path == "/_kl/compact" && req.method == "POST") {
      uint64_t at = 0;
      for_each_store([&](const std::string&, TypeStore& ts) {
        StoreLock lk(ts.seq, ts.seq_stats);
        at = rv.load();
        ts.compacted_rv = at;
        ts.history.clear();
      });
      w.send_json(200, Value::object({{"compacted_rv", static_cast<unsigned long long>(at)}}).dump());
      return;
    }
    if (req.path == "/_kl/drop-watches" && req.method == "POST") {
      size_t n = 0;
      for_each_store([&](const std::string&, TypeStore& ts) {
        std::lock_guard<std::mutex> wg(ts.watches_mu);
        n += ts.watches.size();
        for (const auto& ws : ts.watches) ws->close();
      });
      w.send_json(200, Value::object({{"dropped", static_cast<unsigned long long>(n)}}).dump());
      return;
    }
    if (req.path == "/_kl/stats") {
      Value counts = Value::object();
      Value locks = Value::object();
      size_t total = 0, n_watches = 0;
      uint64_t acq = 0, contended = 0, wait_ns = 0, hold_ns = 0;
      for_each_store([&](const std::string& key, TypeStore& ts) {
        {
          AllShards lk(ts, false);
          size_t n = 0;
          for (auto& sh : ts.shards) n += sh.objs.size();
          counts[key] = static_cast<unsigned long long>(n);
          total += n;
        }
        {
          std::lock_guard<std::mutex> wg(ts.watches_mu);
          n_watches += ts.watches.size();
        }
        // shard locks and the commit-order lock (seq) together; by type, each on its own
        auto account = [](const LockStats& st) {
          return Value::object({{"acquisitions", static_cast<unsigned long long>(st.acquisitions.load())},
                                {"contended", static_cast<unsigned long long>(st.contended.load())},
                                {"wait_ms", static_cast<double>(st.wait_ns.load()) * 1e-6},
                                {"hold_ms", static_cast<double>(st.hold_ns.load()) * 1e-6}});
        };
        for (const LockStats* st : {&ts.stats, &ts.seq_stats}) {
          acq += st->acquisitions.load();
          hold_ns += st->hold_ns.load();
          contended += st->contended.load();
          wait_ns += st->wait_ns.load();
        }
        const uint64_t a = ts.stats.acquisitions.load() + ts.seq_stats.acquisitions.load();
        if (a) {
          // "hold_ms": the serialized part, the commit-order section (what bounds a type's
          // commit rate); "shards": the per-object locks
          locks[key] = Value::object({{"acquisitions", static_cast<unsigned long long>(a)},
                                      {"hold_ms", static_cast<double>(ts.seq_stats.hold_ns.load()) * 1e-6},
                                      {"seq", account(ts.seq_stats)},
                                      {"shards", account(ts.stats)}});
        }
      });
      w.send_json(200, Value::object({{"resourceVersion", static_cast<unsigned long long>(rv.load())},
                                      {"objects", static_cast<unsigned long long>(total)},
                                      {"watches", static_cast<unsigned long long>(n_watches)},
                                      {"requests", static_cast<unsigned long long>(requests.load())},
                                      {"faults_hit", static_cast<unsigned long long>(faults_hit.load())},
                                      {"list_pages", static_cast<unsigned long long>(list_pages.load())},
                                      {"resource_version", rv_str(rv.load())},
                                      {"gc_collected", static_cast<unsigned long long>(gc_collected.load())},
                                      {"store_shards", static_cast<unsigned long long>(opts.store_shards)},
                                      {"gc_pending", static_cast<unsigned long long>([&] {
                                         std::lock_guard<std::mutex> g(gc_mu);
                                         return gc_queue.size();
                                       }())},
                                      // summed over the per-type store locks; by_type_lock has the split
                                      {"store_lock", Value::object({
                                          {"acquisitions", static_cast<unsigned long long>(acq)},
                                          {"contended", static_cast<unsigned long long>(contended)},
                                          {"wait_ms", static_cast<double>(wait_ns) * 1e-6},
                                          {"hold_ms", static_cast<double>(hold_ns) * 1e-6}})},
                                      {"by_type_lock", locks},
                                      {"requests_by_kind", [&] {
                                         Value rq = Value::object();
                                         std::lock_guard<std::mutex> g(req_count_mu);
                                         for (auto& [k, v] : req_counts) rq[k] = static_cast<unsigned long long>(v);
                                         return rq;
                                       }()},
                                      {"by_type", counts}}).dump());
      return;
    }
    w.send(404, "not found\n");
  }

  // ---------------------------------------------------------------- dispatch
  // Request accounting by "METHOD resource[/sub][ watch] code" (exported in /_kl/stats).
  std::mutex req_count_mu;
  std::map<std::string, uint64_t> req_counts;

  void handle(http::Request& req, http::ResponseWriter& w_conn) {
    http::ResponseWriter* wp = &w_conn;  // the response hold's writer, when a fault asks for one
    std::optional<HoldingWriter> holder;
    http::ResponseWriter& w_count = w_conn;
    requests.fetch_add(1, std::memory_order_relaxed);
    std::string res_key = "-";
    struct Count {
      Impl* im;
      const http::Request& req;
      http::ResponseWriter& w;
      std::string& res;
      ~Count() {
        std::string k = req.method + " " + res + " " + std::to_string(w.status_code());
        std::lock_guard<std::mutex> g(im->req_count_mu);
        im->req_counts[k]++;
      }
    } count{this, req, w_count, res_key};
    // trace (core/trace.h): request received ... response sent, per traced object
    struct TraceSpan {
      int64_t t_recv = 0;
      ~TraceSpan() {
        if (!t_trace_tag.empty() && !t_trace_name.empty()) {
          trace::mark_at(t_trace_name, t_trace_tag + ".recv", t_recv);
          trace::mark(t_trace_name, t_trace_tag + ".resp");
        }
        t_trace_tag.clear();
        t_trace_name.clear();
      }
    } span;
    if (trace::armed()) span.t_recv = metrics::now_ns();
    try {
      int hold_ms = 0;
      if (inject_fault(req, w_conn, &hold_ms)) return;
      if (hold_ms > 0 && req.method != "GET") wp = &holder.emplace(w_conn, hold_ms);
      http::ResponseWriter& w = *wp;
      UserInfo user = authenticate(req);
      if (req.path == "/apis/authentication.k8s.io/v1/selfsubjectreviews" && req.method == "POST") {
        // `kubectl auth whoami`: who the request authenticated as
        Value ui = Value::object({{"username", user.username}});
        if (!user.uid.empty()) ui["uid"] = user.uid;
        Value groups = Value::array();
        for (const auto& g : user.groups) groups.push_back(g);
        ui["groups"] = groups;
        w.send_json(201, Value::object({{"kind", "SelfSubjectReview"},
                                        {"apiVersion", "authentication.k8s.io/v1"},
                                        {"metadata", Value::object({{"creationTimestamp", Value()}})},
                                        {"status", Value::object({{"userInfo", ui}})}}).dump());
        return;
      }
      if (req.path == "/api" || req.path == "/apis") {
        discovery(req.path, w);
        return;
      }
      ParsedPath p;
      std::string group, version;
      std::vector<std::string> rest;
      if (!parse_path(req.path, p, group, version, rest)) {
        discovery(req.path, w);
        return;
      }
      res_key = p.ti->rt.plural + (p.sub.empty() ? "" : "/" + p.sub);
      if (p.collection && req.method == "GET") {
        std::string wq = req.query_param("watch");
        if (wq == "1" || wq == "true") res_key += " watch";
      }
      if (span.t_recv && req.method != "GET") {
        t_trace_tag = "kl." + res_key + "." + req.method + "." + field_manager(req, "unknown");
        t_trace_name = p.name;  // a create names its object in the body: do_create sets it
      }
      if (!p.sub.empty() && p.sub != "status") throw StatusError(404, "NotFound", "subresource not supported: " + p.sub);
      if (!p.sub.empty() && !p.ti->rt.has_status) throw StatusError(404, "NotFound", "the server could not find the requested resource");
      const std::string& m = req.method;
      // etcd model: a write is visible (response, watch event) only after a storage
      // commit round trip.  Writes wait concurrently, as they pipeline through raft.
      if (const int64_t lat = write_latency_us.load(std::memory_order_relaxed); lat > 0 && m != "GET") {
        std::this_thread::sleep_for(std::chrono::microseconds(lat));
      }
      if (p.collection) {
        if (m == "GET") {
          std::string wq = req.query_param("watch");
          if (wq == "1" || wq == "true") do_watch(p, req, w);
          else do_list(p, req, w);
        } else if (m == "POST") {
          do_create(p, req, user, w);
        } else {
          throw StatusError(405, "MethodNotAllowed", "method not allowed");
        }
        return;
      }
      if (m == "GET") do_get(p, w, wants_metadata(req));
      else if (m == "PUT") do_update(p, req, user, w);
      else if (m == "PATCH") do_patch(p, req, user, w);
      else if (m == "DELETE") do_delete(p, req, user, w);
      else throw StatusError(405, "MethodNotAllowed", "method not allowed");
    } catch (const StatusError& e) {
      if (!wp->sent()) wp->send_json(e.code, status_body(e.code, e.reason, e.what(), e.details).dump());
    } catch (const std::exception& e) {
      if (!wp->sent()) wp->send_json(500, status_body(500, "InternalError", e.what()).dump());
    }
  }
};

ApiServer::ApiServer(Options o) : impl_(std::make_unique<Impl>(std::move(o))) {}
ApiServer::~ApiServer() { stop(); }

void ApiServer::start() {
  http::ServerOptions so;
  so.addr = impl_->opts.addr;
  so.port = impl_->opts.port;
  so.name = "apiserver";
  so.idle_timeout_ms = 300000;
  if (!impl_->opts.tls_cert_file.empty()) {
    so.tls = net::TlsContext::server_from_files(
        impl_->opts.tls_cert_file, impl_->opts.tls_key_file,
        impl_->opts.client_ca_file.empty() ? "" : net::read_file(impl_->opts.client_ca_file));
  }
  impl_->server = std::make_unique<http::Server>(so);
  Impl* im = impl_.get();
  metrics::set_debug_endpoints(true);  // a test fixture: the bench reads its webhook samples
  http::add_standard_routes(*impl_->server);
  impl_->server->handle("GET", "/healthz", [](http::Request&, http::ResponseWriter& w) { w.send(200, "ok"); });
  impl_->server->handle("GET", "/readyz", [](http::Request&, http::ResponseWriter& w) { w.send(200, "ok"); });
  impl_->server->handle("GET", "/livez", [](http::Request&, http::ResponseWriter& w) { w.send(200, "ok"); });
  impl_->server->handle("GET", "/version", [](http::Request&, http::ResponseWriter& w) {
    w.send_json(200, Value::object({{"major", "1"}, {"minor", "26"}, {"gitVersion", "v1.26.0-kube-lite"}, {"platform", "linux/amd64"}}).dump());
  });
  impl_->server->handle_prefix("/api", [im](http::Request& r, http::ResponseWriter& w) { im->handle(r, w); });
  impl_->server->handle_prefix("/_kl/", [im](http::Request& r, http::ResponseWriter& w) { im->control(r, w); });
  impl_->server->start();
}

uint16_t ApiServer::port() const { return impl_->server ? impl_->server->port() : 0; }

void ApiServer::stop() {
  if (impl_ && impl_->server) {
    impl_->for_each_store([](const std::string&, TypeStore& ts) {
      std::lock_guard<std::mutex> wg(ts.watches_mu);
      for (const auto& ws : ts.watches) ws->close();
    });
    impl_->server->stop(std::chrono::milliseconds(2000));
    impl_->server.reset();
  }
}

}  // namespace bgc::apiserver

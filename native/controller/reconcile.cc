#include "controller/reconcile.h"

#include <algorithm>
#include <cctype>
#include <exception>
#include <optional>
#include <random>
#include <iterator>
#include <future>

#include "core/log.h"
#include "core/metrics.h"
#include "core/trace.h"
#include "kube/quantity.h"

namespace bgc::controller {

// A create refused because the tenant's old Namespace is still terminating (a UserBootstrap
// deleted and created again before the namespace controller finished): expected, and over
// once the Namespace's DELETED event re-queues the tenant, so not reported as a failure.
static bool namespace_terminating(const std::exception& err) {
  const auto* api = dynamic_cast<const kube::ApiError*>(&err);
  if (!api || api->code() != 403) return false;
  for (const auto& c : api->status().get("details").get("causes").items()) {
    if (c.get_string("reason") == "NamespaceTerminating") return true;
  }
  return api->message().find("because it is being terminated") != std::string::npos;
}

using json::Value;
namespace types = kube::types;

Config Config::from_env(const EnvConfig& env) {
  Config c;
  c.listen_addr = env.str("listen_addr");
  c.listen_port = env.u16("listen_port");
  c.workers = static_cast<int>(env.u64_or("workers", 8));
  c.skip_unchanged = env.boolean_or("skip_unchanged", true);
  c.parallel_children = env.boolean_or("parallel_children", true);
  c.child_delete_delay_ms = static_cast<int64_t>(env.u64_or("child_delete_delay_ms", 50));
  c.debounce_ms = static_cast<int64_t>(env.u64_or("debounce_ms", 0));
  c.requeue_secs = static_cast<int64_t>(env.u64_or("requeue_secs", 30));
  c.resync_secs = static_cast<int64_t>(env.u64_or("resync_secs", 300));
  c.error_requeue_ms = static_cast<int64_t>(env.u64_or("error_requeue_ms", 3000));
  c.error_backoff_base_ms = static_cast<int64_t>(env.u64_or("error_backoff_base_ms", 0));
  c.label_children = env.boolean_or("label_children", true);
  c.metadata_watches = env.boolean_or("metadata_watches", true);
  c.events = env.boolean_or("events", true);
  c.projected_watch = env.boolean_or("projected_watch", true);
  c.lease = kube::LeaseSettings::from_env(env, "bacchus-gpu-controller");
  return c;
}

Value controller_owner_ref(const Value& ub) {
  const Value& meta = ub.get("metadata");
  if (!meta.get("uid").is_string() || !meta.get("name").is_string()) {
    throw std::runtime_error("missing object key: .metadata.uid");
  }
  // kube `controller_owner_ref`: apiVersion, kind, name, uid, controller=true
  // (blockOwnerDeletion unset), serialized in k8s-openapi field order.
  return Value::object({{"apiVersion", "bacchus.io/v1"},
                        {"controller", true},
                        {"kind", "UserBootstrap"},
                        {"name", meta.get_string("name")},
                        {"uid", meta.get_string("uid")}});
}

const json::Projection& user_bootstrap_event_projection() {
  using P = json::Projection;
  static const P kMeta[] = {{"name", P::Keep},          {"namespace", P::Keep},  {"uid", P::Keep},
                            {"resourceVersion", P::Keep}, {"generation", P::Keep}, {"deletionTimestamp", P::Keep}};
  // the apiserver's own output: unnamed members are skipped structurally and left out
  static const P kObject[] = {{"apiVersion", P::Keep},
                              {"kind", P::Keep},
                              {"metadata", P::Descend, kMeta, std::size(kMeta), true},
                              {"spec", P::Keep},
                              {"status", P::Keep}};
  static const P kEvent[] = {{"type", P::Keep}, {"object", P::Descend, kObject, std::size(kObject), true}};
  static const P kRoot{"", P::Descend, kEvent, std::size(kEvent), true};
  return kRoot;
}

const json::Projection& child_event_projection() {
  using P = json::Projection;
  static const P kMeta[] = {{"name", P::Keep},
                            {"namespace", P::Keep},
                            {"resourceVersion", P::Keep},
                            {"ownerReferences", P::Keep},
                            {"deletionTimestamp", P::Keep}};
  static const P kObject[] = {{"apiVersion", P::Keep}, {"kind", P::Keep},
                              {"metadata", P::Descend, kMeta, std::size(kMeta), true}};
  static const P kEvent[] = {{"type", P::Keep}, {"object", P::Descend, kObject, std::size(kObject), true}};
  static const P kRoot{"", P::Descend, kEvent, std::size(kEvent), true};
  return kRoot;
}

std::string child_label_selector() { return std::string(kManagedByLabel) + "=" + kManagedByValue; }

// The bodies are written straight into JSON text: a reconcile plans up to four children
// and the only trees it needs are the user's own subtrees (quota, role, rolebinding),
// which are already parsed.  Member order matches what a json::Value build would emit.
std::vector<DesiredChild> desired_children(const Value& ub, bool label) {
  const Value& meta_v = ub.get("metadata");
  const Value& name_v = meta_v.get("name");
  if (!name_v.is_string()) throw std::runtime_error("missing object key: .metadata.name");
  if (!meta_v.get("uid").is_string()) throw std::runtime_error("missing object key: .metadata.uid");
  std::string name = name_v.as_string();
  for (auto& ch : name) ch = static_cast<char>(std::tolower(static_cast<unsigned char>(ch)));
  // kube `controller_owner_ref` (see controller_owner_ref above), as text
  std::string oref = "{\"apiVersion\":\"bacchus.io/v1\",\"controller\":true,\"kind\":\"UserBootstrap\",\"name\":";
  json::escape_string(name_v.as_string(), oref);
  oref += ",\"uid\":";
  json::escape_string(meta_v.get("uid").as_string(), oref);
  oref += "}";
  std::string qname;
  json::escape_string(name, qname);
  const std::string label_json =
      std::string("{") + json::quote(kManagedByLabel) + ":" + json::quote(kManagedByValue) + "}";
  // {"name":..,"ownerReferences":[..](,"labels":{..})}
  std::string meta = "{\"name\":" + qname + ",\"ownerReferences\":[" + oref + "]";
  if (label) meta += ",\"labels\":" + label_json;
  meta += "}";
  auto head = [&](const char* api_version, const char* kind) {
    std::string b;
    b.reserve(256 + meta.size());
    b += "{\"apiVersion\":\"";
    b += api_version;
    b += "\",\"kind\":\"";
    b += kind;
    b += "\",\"metadata\":";
    b += meta;
    return b;
  };
  std::vector<DesiredChild> out;
  // (1) Namespace (controller.rs:69-87)
  out.push_back({&types::Namespace, "", name, head("v1", "Namespace") + "}"});
  const Value& spec = ub.get("spec");
  // (2) ResourceQuota (controller.rs:89-110)
  if (const Value* q = spec.find("quota"); q && !q->is_null()) {
    std::string b = head("v1", "ResourceQuota");
    b += ",\"spec\":";
    q->dump_to(b);
    b += "}";
    out.push_back({&types::ResourceQuota, name, name, std::move(b)});
  }
  // (3) Role: the user's object with ownerReferences overwritten (controller.rs:112-124)
  if (const Value* r = spec.find("role"); r && !r->is_null()) {
    Value role = Value::object({{"apiVersion", "rbac.authorization.k8s.io/v1"}, {"kind", "Role"}});
    Value m = r->get("metadata").is_object() ? r->get("metadata") : Value::object();
    m["ownerReferences"] = Value::array({controller_owner_ref(ub)});
    if (label) {
      if (!m.get("labels").is_object()) m["labels"] = Value::object();
      m["labels"][kManagedByLabel] = kManagedByValue;
    }
    role["metadata"] = m;
    if (const Value* rules = r->find("rules"); rules && !rules->is_null()) role["rules"] = *rules;
    // The URL name is the namespace name; a Role whose metadata.name differs is
    // rejected by the apiserver on every reconcile, exactly like the reference (Q9).
    out.push_back({&types::Role, name, name, role.dump()});
  }
  // (4) RoleBinding, gated on status.synchronized_with_sheet (controller.rs:126-152)
  if (const Value* rb = spec.find("rolebinding"); rb && !rb->is_null()) {
    const Value& st = ub.get("status");
    if (st.is_object() && st.get("synchronized_with_sheet").is_bool() && st.get("synchronized_with_sheet").as_bool()) {
      std::string b = head("rbac.authorization.k8s.io/v1", "RoleBinding");
      b += ",\"roleRef\":";
      rb->get("role_ref").dump_to(b);
      if (const Value* sub = rb->find("subjects"); sub && !sub->is_null()) {
        b += ",\"subjects\":";
        sub->dump_to(b);
      }
      b += "}";
      out.push_back({&types::RoleBinding, name, name, std::move(b)});
    }
  }
  return out;
}

Reconciler::Reconciler(kube::KubeClient& client, kube::Controller& ctrl, Config cfg)
    : client_(client), ctrl_(ctrl), cfg_(cfg), pool_(static_cast<size_t>(std::max(4, cfg.workers * 3)), "apply") {}

Reconciler::Stats Reconciler::stats() const {
  return {stats_applied_.load(std::memory_order_relaxed), stats_skipped_.load(std::memory_order_relaxed),
          stats_verified_.load(std::memory_order_relaxed), stats_repaired_.load(std::memory_order_relaxed)};
}

static std::string lower(std::string s) {
  for (auto& ch : s) ch = static_cast<char>(std::tolower(static_cast<unsigned char>(ch)));
  return s;
}

// Every record of one tenant (its children's applies, its fast-path state, its failure
// count) lives in the shard of its namespace name: the lower-cased UserBootstrap name,
// which is also each child's name (the Namespace) or namespace (the rest).
Reconciler::Shard& Reconciler::shard(const std::string& ns_name) const {
  return shards_[std::hash<std::string>{}(ns_name) % kShards];
}

static std::string child_key(const DesiredChild& c) { return c.rt->plural + "/" + c.ns + "/" + c.name; }

// Publishes the sizes of the two per-tenant caches (bounded-memory check under churn).
void Reconciler::publish_cache_sizes() {
  static auto& reg = metrics::Registry::global();
  static auto& a = reg.gauge("bgc_controller_apply_cache_entries", "Children with a remembered last apply");
  static auto& o = reg.gauge("bgc_controller_owner_state_entries", "UserBootstraps with fast-path state");
  a.set(static_cast<double>(applied_entries_.load(std::memory_order_relaxed)));
  o.set(static_cast<double>(owner_entries_.load(std::memory_order_relaxed)));
}

void Reconciler::erase_applied_locked(Shard& sh, const std::string& key) {
  if (sh.last_applied.erase(key)) applied_entries_.fetch_sub(1, std::memory_order_relaxed);
}

void Reconciler::erase_owner_state_locked(Shard& sh, const std::string& owner) {
  if (sh.ub_state.erase(owner)) owner_entries_.fetch_sub(1, std::memory_order_relaxed);
}

void Reconciler::forget(const kube::ResourceType& rt, const Value& child) {
  const std::string ns = kube::meta_namespace(child), name = kube::meta_name(child);
  Shard& sh = shard(ns.empty() ? name : ns);
  {
    std::lock_guard<std::mutex> lk(sh.mu);
    const std::string key = rt.plural + "/" + ns + "/" + name;
    erase_applied_locked(sh, key);
    if (auto a = sh.applying.find(key); a != sh.applying.end()) a->second = true;
    for (const auto& ref : child.get("metadata").get("ownerReferences").items()) {
      if (ref.get_string("kind") == types::UserBootstrap.kind) erase_owner_state_locked(sh, ref.get_string("name"));
    }
  }
  publish_cache_sizes();
}

void Reconciler::forget_owner_locked(Shard& sh, const std::string& owner) {
  sh.failures.erase(owner);
  const std::string ns = lower(owner);
  erase_owner_state_locked(sh, owner);
  auto drop = [&](const std::string& key) {
    erase_applied_locked(sh, key);
    if (auto a = sh.applying.find(key); a != sh.applying.end()) a->second = true;
  };
  drop(types::Namespace.plural + "//" + ns);
  for (const auto* rt : {&types::ResourceQuota, &types::Role, &types::RoleBinding}) drop(rt->plural + "/" + ns + "/" + ns);
}

void Reconciler::forget_owner(const std::string& owner) {
  Shard& sh = shard(lower(owner));
  {
    std::lock_guard<std::mutex> lk(sh.mu);
    forget_owner_locked(sh, owner);
  }
  publish_cache_sizes();
}

bool Reconciler::owner_live(const std::string& name, const std::string& uid) {
  kube::ObjPtr cur = ctrl_.store().get("", name);
  return cur && cur->get("metadata").get_string("uid") == uid;
}

bool Reconciler::fresh(const std::string& owner_name, const std::string& owner_rv) {
  std::vector<ChildRef> children;
  {
    Shard& sh = shard(lower(owner_name));
    std::lock_guard<std::mutex> lk(sh.mu);
    auto it = sh.ub_state.find(owner_name);
    if (it == sh.ub_state.end() || it->second.owner_rv != owner_rv) return false;
    children = it->second.children;
  }
  for (const auto& c : children) {
    kube::Store* store = ctrl_.child_store(c.rt->plural);
    if (!store) return false;
    kube::ObjPtr cur = store->get(c.ns, c.name);
    if (!cur || kube::meta_rv(*cur) != c.rv) return false;
  }
  return true;
}

size_t Reconciler::cached_children() const { return applied_entries_.load(std::memory_order_relaxed); }

bool Reconciler::is_own_write(const kube::ResourceType& rt, const Value& child) const {
  if (!cfg_.skip_unchanged) return false;
  const std::string ns = kube::meta_namespace(child), name = kube::meta_name(child);
  const std::string key = rt.plural + "/" + ns + "/" + name;
  Shard& sh = shard(ns.empty() ? name : ns);
  std::lock_guard<std::mutex> lk(sh.mu);
  auto it = sh.last_applied.find(key);
  return it != sh.last_applied.end() && it->second.rv == kube::meta_rv(child);
}

// Up to date: the same body as our last apply, and the watch cache shows that apply's
// result — or still shows exactly what it showed when we applied (absent, or the version
// before), i.e. our write's watch echo is on its way.  Watch events arrive in order, so
// anything another writer did after our apply reaches the cache after that echo and is
// seen by a later reconcile; without this a reconcile that overtakes the echo (the status
// write right after the quota apply) re-applies an unchanged ResourceQuota.
bool Reconciler::up_to_date(const DesiredChild& c, const std::string& body_hash) {
  if (!cfg_.skip_unchanged) return false;
  kube::Store* store = ctrl_.child_store(c.rt->plural);
  if (!store) return false;
  kube::ObjPtr cur = store->get(c.ns, c.name);
  Shard& sh = shard(c.name);
  std::lock_guard<std::mutex> lk(sh.mu);
  auto it = sh.last_applied.find(child_key(c));
  if (it == sh.last_applied.end() || it->second.body_hash != body_hash) return false;
  const Applied& a = it->second;
  const std::string rv = cur ? kube::meta_rv(*cur) : std::string();
  if (cur && rv == a.rv) return true;
  // The echo is in flight only briefly (milliseconds): past that, a cache that still shows
  // the old state means the object changed or went away in a way whose events arrived
  // before our record of the apply (e.g. created and deleted again meanwhile).
  if (std::chrono::steady_clock::now() - a.at > std::chrono::seconds(2)) return false;
  return cur ? (a.prev_present && rv == a.prev_rv) : !a.prev_present;
}

void Reconciler::apply_child(const DesiredChild& c, const std::string& body_hash, const std::string& body_json) {
  static auto& applied = metrics::Registry::global().counter("bgc_apply_total", "Server-side applies issued");
  static auto& dropped = metrics::Registry::global().counter(
      "bgc_apply_records_dropped_total", "Applies whose result was not recorded: the child was deleted while in flight");
  kube::Store* store = ctrl_.child_store(c.rt->plural);
  const std::string key = child_key(c);
  Shard& sh = shard(c.name);
  {
    std::lock_guard<std::mutex> lk(sh.mu);
    sh.applying[key] = false;
  }
  // A watch event of this child can be processed at any point from here on (the apply's
  // own ADDED, then a DELETED when someone removes it at once).  The cache state read now
  // is what the "echo pending" rule of up_to_date compares against, so a forget() of the
  // child before the result is recorded must void the record (Shard::applying).
  struct Unmark {
    Shard& sh;
    const std::string& key;
    bool armed = true;
    ~Unmark() {
      if (!armed) return;
      std::lock_guard<std::mutex> lk(sh.mu);
      sh.applying.erase(key);
    }
  } unmark{sh, key};
  const kube::ObjPtr before = store ? store->get(c.ns, c.name) : nullptr;
  const bool traced = trace::armed();
  if (traced) trace::mark(c.name, "ctl.apply." + c.rt->plural + ".send");
  std::string rv = client_.apply_rv(*c.rt, c.ns, c.name, body_json, kFieldManager, /*force=*/true);
  if (traced) trace::mark(c.name, "ctl.apply." + c.rt->plural + ".done");
  applied.inc();
  if (after_apply_) after_apply_(c);
  {
    std::lock_guard<std::mutex> lk(sh.mu);
    unmark.armed = false;
    auto a = sh.applying.find(key);
    const bool forgotten = a != sh.applying.end() && a->second;
    if (a != sh.applying.end()) sh.applying.erase(a);
    if (forgotten) {
      dropped.inc();  // the next reconcile (queued by that DELETED event) applies again
    } else {
      auto [it, inserted] = sh.last_applied.try_emplace(key);
      it->second = {body_hash, std::move(rv), before ? kube::meta_rv(*before) : std::string(), before != nullptr,
                    std::chrono::steady_clock::now()};
      if (inserted) applied_entries_.fetch_add(1, std::memory_order_relaxed);
    }
  }
  publish_cache_sizes();
  stats_applied_.fetch_add(1, std::memory_order_relaxed);
}

// SSA-shaped coverage: every member `want` sets is in `have` with a covered value.  Maps
// may hold more (other managers' fields survive a forced apply); ownerReferences is keyed
// by uid (each wanted reference must be present); other lists are atomic (same length,
// element by element), as a forced apply replaces them.  A ResourceQuota's `hard` values
// are quantities, compared by value: the apiserver stores them canonical ("1000m" -> "1").
static bool covers(const Value& want, const Value& have, std::string_view key = {}, bool quantities = false) {
  if (want.is_object()) {
    if (!have.is_object()) return false;
    const auto& keys = want.keys();
    const auto& vals = want.values();
    for (size_t i = 0; i < keys.size(); ++i) {
      const Value* h = have.find(keys[i]);
      if (!h || !covers(vals[i], *h, keys[i], key == "hard")) return false;
    }
    return true;
  }
  if (quantities && want.is_string() && have.is_string() && want.as_string() != have.as_string()) {
    return kube::same_quantity(want.as_string(), have.as_string());
  }
  if (want.is_array()) {
    if (!have.is_array()) return false;
    const auto& w = want.items();
    const auto& h = have.items();
    if (key == "ownerReferences") {
      for (const auto& x : w) {
        if (std::none_of(h.begin(), h.end(), [&](const Value& y) { return covers(x, y); })) return false;
      }
      return true;
    }
    if (w.size() != h.size()) return false;
    for (size_t i = 0; i < w.size(); ++i) {
      if (!covers(w[i], h[i])) return false;
    }
    return true;
  }
  return want == have;
}

bool Reconciler::verified_in_sync(const DesiredChild& c, const std::string& body_hash) {
  static auto& reg = metrics::Registry::global();
  static auto& checked = reg.counter("bgc_resync_checks_total", "Children read back from the apiserver by a resync");
  static auto& drifted = reg.counter("bgc_resync_repairs_total", "Children a resync found drifted or missing (re-applied)");
  checked.inc();
  stats_verified_.fetch_add(1, std::memory_order_relaxed);
  std::optional<Value> live = client_.get_opt(*c.rt, c.ns, c.name);
  if (live && covers(json::parse(c.body), *live)) {
    const std::string rv = kube::meta_rv(*live);
    Shard& sh = shard(c.name);
    std::lock_guard<std::mutex> lk(sh.mu);
    auto [it, inserted] = sh.last_applied.try_emplace(child_key(c));
    it->second = {body_hash, rv, rv, true, std::chrono::steady_clock::now()};
    if (inserted) applied_entries_.fetch_add(1, std::memory_order_relaxed);
    return true;
  }
  drifted.inc();
  stats_repaired_.fetch_add(1, std::memory_order_relaxed);
  LOG_INFO("controller") << "resync: " << c.rt->kind << " " << (c.ns.empty() ? "" : c.ns + "/") << c.name
                         << (live ? " drifted" : " missing") << "; re-applying";
  return false;
}

bool Reconciler::resync_due(const std::string& owner_name) {
  if (!cfg_.skip_unchanged || cfg_.resync_secs <= 0) return false;
  Shard& sh = shard(lower(owner_name));
  std::lock_guard<std::mutex> lk(sh.mu);
  auto it = sh.ub_state.find(owner_name);
  return it != sh.ub_state.end() && std::chrono::steady_clock::now() >= it->second.next_resync;
}

std::chrono::steady_clock::time_point Reconciler::next_resync_time() {
  // spread over [0.75, 1] of the period: UserBootstraps reconciled together (a restart, a
  // bulk import) do not all come due in the same second
  thread_local std::minstd_rand rng{std::random_device{}()};
  const int64_t period_ms = cfg_.resync_secs * 1000;
  const int64_t ms = period_ms - static_cast<int64_t>(rng() % static_cast<uint64_t>(period_ms / 4 + 1));
  return std::chrono::steady_clock::now() + std::chrono::milliseconds(ms);
}

kube::Action Reconciler::reconcile(const kube::ObjPtr& ub_ptr) {
  auto& reg = metrics::Registry::global();
  static auto& hist = reg.histogram("bgc_reconcile_duration_seconds", "Wall time of one reconcile");
  static auto& ok = reg.counter("bgc_reconcile_total", "Reconciles", {{"result", "ok"}});
  static auto& failed = reg.counter("bgc_reconcile_total", "Reconciles", {{"result", "error"}});
  // bgc_reconcile_total is counted in the sample log's critical section (SampleLog::add), so
  // the samples of a bench window are exactly that counter's increments over the window.
  static auto& ring = [&]() -> metrics::SampleLog& {
    auto& r = reg.samples("reconcile");
    r.link("bgc_reconcile_total{result=\"ok\"}", &ok);
    r.link("bgc_reconcile_total{result=\"error\"}", &failed);
    return r;
  }();
  static auto& skipped = reg.counter("bgc_apply_skipped_total", "Applies skipped: child already as last written");
  struct Timed {
    const int64_t t0 = metrics::now_ns();
    const int exceptions = std::uncaught_exceptions();
    ~Timed() {
      const double e = static_cast<double>(metrics::now_ns() - t0) * 1e-9;
      hist.observe(e);
      ring.add(e, std::uncaught_exceptions() > exceptions ? &failed : &ok);  // thrown: error_policy runs next
    }
  } timed;
  const Value& ub = *ub_ptr;
  const std::string owner_name = kube::meta_name(ub), owner_rv = kube::meta_rv(ub);
  // The periodic requeue normally trusts the watch cache; once per resync period it reads
  // the children back from the apiserver instead.
  const bool verify = resync_due(owner_name);
  if (!verify && cfg_.skip_unchanged && fresh(owner_name, owner_rv)) {
    static auto& fast = reg.counter("bgc_reconcile_fast_total", "Reconciles with UB and children unchanged since the last one");
    fast.inc();
    return kube::Action::requeue_after(std::chrono::milliseconds(cfg_.requeue_secs * 1000));
  }
  std::vector<DesiredChild> children = desired_children(ub, cfg_.label_children);
  LOG_INFO("controller") << "reconciling " << children.front().name;

  std::vector<std::string> hashes;
  hashes.reserve(children.size());
  for (const auto& c : children) hashes.push_back(std::to_string(std::hash<std::string>{}(c.body)));

  auto run_one = [&](size_t i) {
    if (verify ? verified_in_sync(children[i], hashes[i]) : up_to_date(children[i], hashes[i])) {
      skipped.inc();
      stats_skipped_.fetch_add(1, std::memory_order_relaxed);
      return;
    }
    try {
      apply_child(children[i], hashes[i], children[i].body);
    } catch (const std::exception& e) {
      if (!namespace_terminating(e)) {
        LOG_ERROR("controller") << "failed to patch " << children[i].rt->kind << ": " << e.what();
      }
      throw;
    }
  };

  // Stage 1: the Namespace (namespaced children cannot exist before it).
  // Stage 2: ResourceQuota and Role, concurrently (independent objects).
  // Stage 3: the RoleBinding — only after every earlier apply succeeded, so a user is
  //          never bound into a namespace whose quota failed to apply (the reference
  //          gets the same guarantee from its sequential `?` chain).
  // A reconcile can still be running when its UserBootstrap is deleted: forget_owner()
  // then runs first (on the watcher thread) and the applies below would re-insert cache
  // entries that nothing removes.  Every exit re-checks the watch cache under mu_ and
  // drops the owner's entries when the UB (this uid) is gone.
  const std::string owner_uid = ub.get("metadata").get_string("uid");
  Shard& sh = shard(children.front().name);
  try {
    apply_all(children, run_one);
  } catch (...) {
    {
      // A failed apply invalidates what we remember of this tenant's children (e.g. a
      // ResourceQuota refused because its Namespace is gone): the retry re-applies them all.
      std::lock_guard<std::mutex> lk(sh.mu);
      const int failures = sh.failures.count(owner_name) ? sh.failures[owner_name] : 0;
      forget_owner_locked(sh, owner_name);
      if (failures && owner_live(owner_name, owner_uid)) sh.failures[owner_name] = failures;  // keep the backoff
    }
    publish_cache_sizes();
    throw;
  }
  {
    std::lock_guard<std::mutex> lk(sh.mu);
    if (!sh.failures.empty()) sh.failures.erase(owner_name);
    if (!owner_live(owner_name, owner_uid)) {
      forget_owner_locked(sh, owner_name);
    } else if (cfg_.skip_unchanged) {
      UbState st;
      st.owner_rv = owner_rv;
      bool complete = true;
      for (const auto& c : children) {
        auto it = sh.last_applied.find(child_key(c));
        if (it == sh.last_applied.end()) {
          complete = false;
          break;
        }
        st.children.push_back({c.rt, c.ns, c.name, it->second.rv});
      }
      if (complete) {
        auto [it, inserted] = sh.ub_state.try_emplace(owner_name);
        // a verification pass restarts the period; otherwise the pending one carries over
        st.next_resync = verify || inserted ? next_resync_time() : it->second.next_resync;
        it->second = std::move(st);
        if (inserted) owner_entries_.fetch_add(1, std::memory_order_relaxed);
      }
    }
  }
  publish_cache_sizes();
  return kube::Action::requeue_after(std::chrono::milliseconds(cfg_.requeue_secs * 1000));
}

void Reconciler::apply_all(const std::vector<DesiredChild>& children, const std::function<void(size_t)>& run_one) {
  run_one(0);
  std::vector<size_t> middle, last;
  for (size_t i = 1; i < children.size(); ++i) {
    (children[i].rt == &types::RoleBinding ? last : middle).push_back(i);
  }
  if (cfg_.parallel_children && middle.size() > 1) {
    std::vector<std::future<void>> futs;
    for (size_t i : middle) futs.push_back(pool_.submit([&, i] { run_one(i); }));
    std::exception_ptr first;
    for (auto& f : futs) {
      try {
        f.get();
      } catch (...) {
        if (!first) first = std::current_exception();
      }
    }
    if (first) std::rethrow_exception(first);
  } else {
    for (size_t i : middle) run_one(i);
  }
  for (size_t i : last) run_one(i);
}

kube::Action Reconciler::error_policy(const kube::ObjPtr& ub, const std::exception& err) {
  const Value& meta = ub->get("metadata");
  if (namespace_terminating(err)) {
    static auto& waits = metrics::Registry::global().counter(
        "bgc_reconcile_namespace_terminating_total", "Reconciles that waited for the tenant's old Namespace to terminate");
    waits.inc();
    LOG_INFO("controller") << "\"" << meta.get_string("name", "<unknown>")
                           << "\": its namespace is still terminating; retrying once it is gone";
    return kube::Action::requeue_after(std::chrono::milliseconds(cfg_.error_requeue_ms));
  }
  LOG_ERROR("controller") << "error reconciling \"" << meta.get_string("namespace", "<unknown>") << "/"
                          << meta.get_string("name", "<unknown>") << "\": " << err.what();
  if (events_) events_->record(kube::types::UserBootstrap, *ub, "Warning", "ReconcileFailed", err.what());
  int64_t delay = cfg_.error_requeue_ms;
  if (cfg_.error_backoff_base_ms > 0) {
    int n;
    {
      const std::string owner = meta.get_string("name");
      Shard& sh = shard(lower(owner));
      std::lock_guard<std::mutex> lk(sh.mu);
      n = ++sh.failures[owner];
      // a UserBootstrap deleted meanwhile (forget_owner may have run already) keeps no count
      if (!owner_live(owner, meta.get_string("uid"))) sh.failures.erase(owner);
    }
    const int shift = std::min(n - 1, 30);
    delay = std::min<int64_t>(cfg_.error_requeue_ms, cfg_.error_backoff_base_ms << shift);
  }
  return kube::Action::requeue_after(std::chrono::milliseconds(delay));
}

}  // namespace bgc::controller

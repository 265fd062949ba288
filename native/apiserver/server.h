// kube-lite: an in-process Kubernetes API server for tests, the bench harness and
// offline e2e runs (north-star component N7; no kind/etcd exist in this environment).
//
// Fidelity targets (what the controller/admission/synchronizer/node-agent rely on):
//  * REST: GET/LIST/WATCH (resourceVersion resume, bookmarks, 410 Gone after compaction),
//    POST, PUT (optimistic concurrency), PATCH (json-patch, merge-patch,
//    strategic-merge as merge, apply-patch+yaml = server-side apply with field managers,
//    conflicts and force), DELETE (finalizers, ownerReference GC, namespace cascade);
//  * status subresource semantics for CRDs and built-ins;
//  * CustomResourceDefinitions registered dynamically, with structural schema
//    validation (422 Invalid);
//  * MutatingWebhookConfiguration callouts over TLS with caBundle verification,
//    JSONPatch responses, timeouts and failurePolicy (the reference's webhook path,
//    charts/.../templates/webhook.yaml:11-27);
//  * static-token authentication (kube-apiserver --token-auth-file format) and
//    impersonation for system:masters;
//  * fault injection (/_kl/faults) and watch compaction/drops for resilience tests.
#pragma once

#include <cstdint>
#include <map>
#include <memory>
#include <string>

namespace bgc::apiserver {

struct Options {
  std::string addr = "127.0.0.1";
  uint16_t port = 0;
  std::string token_file;         // CSV: token,user,uid,"group1,group2"
  bool anonymous_admin = true;    // no token => system:admin in system:masters
  std::string tls_cert_file;      // serve HTTPS when set
  // x509 client-certificate authentication (kube-apiserver --client-ca-file): a verified
  // client certificate authenticates as user CN with groups O when no bearer token is sent
  std::string client_ca_file;
  std::string tls_key_file;
  // "namespace/service" -> "host:port": where a webhook's clientConfig.service is reachable.
  std::map<std::string, std::string> service_overrides;
  size_t history_limit = 50000;  // watch-cache events kept per type for resume (k8s keeps ~100)
  int bookmark_interval_ms = 60000;
  bool validate_schema = true;
  // Label-selector watches see an update that moves an object into their selector as ADDED
  // and one that moves it out as DELETED, as on a real apiserver.  false (kube-lite
  // --no-selector-transitions) drops such events instead: a lost-event scenario.
  bool selector_transitions = true;
  // Namespace deletion as the namespace controller does it: DELETE marks the namespace
  // Terminating, creates in it are refused (403, NamespaceLifecycle), its contents are
  // deleted, then the namespace.  false (--instant-namespace-deletion): removed at once.
  bool namespace_termination = true;
  int max_watch_seconds = 1800;
  // Watch write coalescing: after a wake-up with few events queued, wait this long for
  // more before writing (fewer wake-ups/syscalls per event at high event rates, at the
  // cost of up to this much added delivery latency).  0 = write immediately.
  int watch_coalesce_us = 50;  // measured on MI355X: +7 % CR/s, -6 % CPU/CR, lower p50 (profiles/archive/watch_coalesce_r1/)
  // Garbage-collector threads (cascading deletion of dependents and namespace contents).
  // One thread fell 10-14k deletions behind over 100k tenants at ~10k CR/s on the MI355X
  // box; two keep the backlog at 0 with unchanged CR/s (profiles/archive/gc_workers_r1/).
  int gc_workers = 2;
  // Storage commit latency added to every write (POST/PUT/PATCH/DELETE) before it is
  // applied: a real apiserver answers a write only after etcd's raft commit + fsync
  // (typically 1-10 ms).  0 = in-memory speed.
  int64_t write_latency_us = 0;
  // Opaque resourceVersions ("kl.<base36>" instead of decimal digits): clients must treat
  // them as opaque strings, as the Kubernetes API contract says; this catches any that
  // parse or compare them.
  bool opaque_rv = false;
  // Paginated LIST (limit/continue) serves later pages from a snapshot taken at the first
  // page; continue tokens expire after this long (then 410 Expired, as etcd compaction).
  int continue_ttl_ms = 60000;
  // Webhook callouts: HTTP/1.1 keep-alive pool by default; webhook_http2 offers h2 by ALPN
  // and multiplexes the callouts as streams over webhook_h2_connections connections (as
  // the real apiserver's Go client does over one).  With kube-lite's mutex store lock the
  // HTTP/1.1 pool measured equal or better at N=1..8 (profiles/archive/http2_r2/after_store_lock/).
  bool webhook_http2 = false;
  size_t webhook_h2_connections = 4;
  // HTTP/2 webhook callouts: the calling handler threads read their responses themselves
  // (http::ClientOptions::h2_caller_reads) instead of a reader thread per connection that
  // then wakes them.  Off: on the MI355X box it raised the webhook p50 0.57 -> 0.71 ms (the
  // reader-role hand-offs cost more wake-ups than they save, profiles/kl_shard_r4/
  // caller_reads/).  BGC_KL_H2_CALLER_READS=1 turns it on.
  bool webhook_h2_caller_reads = false;
  // Key-hashed shards of each type's object store, each with its own lock (commits of
  // different objects run in parallel; a commit-order lock per type assigns resourceVersions
  // and queues events).  1 = one lock per type, the round-3 store.  BGC_KL_STORE_SHARDS
  // overrides.
  size_t store_shards = 16;
};

class ApiServer {
 public:
  explicit ApiServer(Options o);
  ~ApiServer();
  void start();
  uint16_t port() const;
  void stop();

  struct Impl;

 private:
  std::unique_ptr<Impl> impl_;
};

}  // namespace bgc::apiserver

// Node-level orchestration of the HIP health diagnostics.
//
// The reference never touches a GPU (its only GPU touch-point is the quota key at
// reference src/synchronizer.rs:268,276); these pieces decide *how* the node agent runs
// the gfx950 checks of gpu/diag.h on a whole 8 x MI355X node:
//
//   * every GPU is diagnosed on its own thread (hipSetDevice is per thread, the diag
//     library keeps its error string thread_local), so a node takes one GPU's wall time
//     instead of eight;
//   * the burn-in is a node-level phase: all GPUs under diagnosis start their sustained
//     MFMA load together behind a start barrier while one sampler reads every GPU, so
//     the node's power delivery and cooling carry the full load at once — the failure a
//     GPU-by-GPU burn never provokes.  The phase is judged on the summed power, the peak
//     hotspot and the slowest GPU against the fastest under that shared load.
//
// DiagEngine is the seam between orchestration and kernels: HipDiagEngine drives
// libbgc_gpu_diag.so; ScriptedDiagEngine replays a mock fixture's "diag_script" (per-GPU
// durations and outcomes) so fencing and concurrency are tested on CPU hosts.
#pragma once

#include <chrono>
#include <cstdint>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "core/cancel.h"
#include "core/json.h"
#include "gpu/device.h"
#include "gpu/diag.h"

namespace bgc::gpu {

struct DiagPlan {
  uint64_t hbm_bytes = 1ULL << 30;       // bandwidth phases (two buffers of this size)
  double hbm_walk_fraction = 0.9;        // address-pattern walk of this share of free VRAM (0 = off)
  uint64_t hbm_walk_chunk_bytes = 4ULL << 30;
  int hbm_walk_budget_ms = 20000;
  uint64_t pcie_bytes = 256ULL << 20;    // 0 = off
  int soak_size = 8192;
  int soak_launches = 20;                // 0 = off
  bool lowp = true;                      // MX fp8 / fp4 matrix-core tiles and rates
  int burn_ms = 0;                       // node-level burn phase (0 = off)
  int burn_dtype = BGC_BURN_BF16;         // its matrix-core path (bf16, MX fp8, MX fp4)
};

class DiagEngine {
 public:
  virtual ~DiagEngine() = default;
  virtual std::string name() const = 0;
  // How far ahead node_burn schedules a common start (time a burn needs to get ready).
  virtual int start_lead_ms() const { return 0; }
  // Everything but the burn for one GPU: {"hbm","hbm_walk","mfma","lowp","gemm","pcie","soak"}.
  // Throws on a HIP/library error.
  virtual json::Value checks(Backend& backend, const GpuInfo& g, int hip_device, const DiagPlan& plan,
                             uint32_t seed) = 0;
  // Sustained MFMA load on one GPU (Diag::burn's result shape; dtype BGC_BURN_*), starting at start_at
  // (steady clock; the epoch = now) so that GPUs burning together start together.
  virtual json::Value burn(int hip_device, int duration_ms, uint32_t seed, int dtype,
                           std::chrono::steady_clock::time_point start_at) = 0;
  // device -> PCI BDF of the GPU it must be (worker engines verify it before running).
  virtual void set_device_bdfs(std::map<int, std::string>) {}
};

// In this process (the python bindings, tools): the first call initialises HIP here.
std::unique_ptr<DiagEngine> make_hip_diag_engine();
// The node agent's engine: every check and burn runs in a child process (`exe
// --diag-worker`, see diag_worker_main) that sees only its own GPU
// (ROCR_VISIBLE_DEVICES).  The agent itself never initialises HIP, so between passes it
// holds no GPU context and no VRAM, a GPU fault in a kernel ends the worker rather than
// the agent, and amdsmi's process list shows only tenants' processes (a container's
// getpid() is not the host PID KFD reports, so the agent could not recognise itself).
// PCIe sections of concurrent workers take turns on an flock(2) of pcie_lock_path.
// A running worker is killed as soon as `cancel` is cancelled (the agent stopping).
std::unique_ptr<DiagEngine> make_process_diag_engine(std::string exe, std::string backend_kind,
                                                     std::string mock_fixture_path, std::string pcie_lock_path,
                                                     const CancelToken* cancel = nullptr);
// PCI addresses of the HIP devices, in HIP order, read by a worker process.
std::vector<std::string> worker_device_bdfs(const std::string& exe);
// `node-agent --diag-worker`: the request JSON in $BGC_DIAG_REQUEST ({"op": "devices" |
// "checks" | "burn", ...}), the result JSON (or {"error": ...}) on stdout.
int diag_worker_main();

json::Value to_json(const DiagPlan& p);
DiagPlan diag_plan_from_json(const json::Value& v);
// Replays backend.diag_script() (re-read on every call):
//   {"checks_ms": 200, "burn_tflops": 2400,
//    "gpus": {"<index>": {"checks_ms": .., "burn_tflops": .., "walk_mismatches": .., "fail": "<text>"}}}
std::unique_ptr<DiagEngine> make_scripted_diag_engine(Backend& backend);

// Host<->device copy rates (Diag::pcie) plus the PCIe link width/speed sampled through
// `backend` while the copies run (links drop to a low-power rate when idle), and the
// link's replay/recovery counter deltas over the test.
json::Value pcie_check(Backend& backend, const GpuInfo& g, int hip_device, uint64_t bytes, uint32_t seed);

// One GPU's burn while a side thread samples it (power, clocks, temperatures, throttle
// residency); the single-GPU form of node_burn.
json::Value burn_in(Backend& backend, int index, int hip_device, int duration_ms, uint32_t seed,
                    DiagEngine* engine = nullptr, int dtype = BGC_BURN_BF16);

struct NodeBurnResult {
  std::vector<json::Value> per_gpu;   // burn section per entry of `which` (burn_in's shape)
  json::Value node;                   // {gpus, power_sum_max_w, power_sum_mean_w, peak_hotspot_c, balance, ...}
};

// All GPUs `which` (indices into gpus; hip_devs[i] is gpus[i]'s HIP device) burn at once
// for duration_ms behind a start barrier.
NodeBurnResult node_burn(Backend& backend, DiagEngine& engine, const std::vector<GpuInfo>& gpus,
                         const std::vector<int>& hip_devs, const std::vector<size_t>& which, int duration_ms,
                         uint32_t seed, int dtype = BGC_BURN_BF16);

// Node-level verdict over a node_burn: adds "failures"/"passed" to the node summary and
// returns, per GPU in the burn, the failures that name it (a GPU far below the node's
// fastest under shared load; every GPU when the node power or hotspot limit is broken).
std::vector<std::vector<std::string>> judge_node_burn(NodeBurnResult& r, const DiagFloors& floors);

// The GPUs' HIP device ids, by PCI BDF when the diag library can name them (HIP renumbers
// visible devices inside a container), else amdsmi's hip_id, else the index.
std::vector<int> hip_devices_for(const std::vector<GpuInfo>& gpus, const std::vector<std::string>& hip_bdfs);

}  // namespace bgc::gpu

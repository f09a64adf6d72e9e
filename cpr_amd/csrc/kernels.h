// Host-visible launchers for the gfx950 kernels in kernels.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "../../include/cpr_hip.h"
#include "bk_lane.h"
#include "ethereum_lane.h"
#include "nakamoto_lane.h"
#include "fc16_lane.h"
#include "summary.h"
#include "ts_lane.h"

// occupancy of the per-lane event-engine kernels (B_k, Ethereum, Tailstorm fused episodes
// and rollouts): they are bound by dependent memory latency, so waves per SIMD matter more
// than the few VGPRs a tighter budget spills. CPR_EV_WAVES = minimum waves per SIMD the
// compiler must allow (0: unconstrained; a translation unit may set its own before including
// this header: kernels_ts.hip 2; Ethereum and B_k unconstrained, as measured in
// profiles/r03f_event_occupancy_ab.log). tools/occupancy_ab.sh builds variants.
#ifndef CPR_EV_WAVES
#define CPR_EV_WAVES 0
#endif
// CPR_EV_SCHED = 1: wave-coherent dispatch of the event engines' work (wave_sched.h);
// 0: one plain event loop per lane (the round-2 kernels), kept for A/B variants
#ifndef CPR_EV_SCHED
#define CPR_EV_SCHED 1
#endif
#if CPR_EV_WAVES > 0
#define CPR_EV_OCC __attribute__((amdgpu_waves_per_eu(CPR_EV_WAVES)))
#else
#define CPR_EV_OCC
#endif

namespace cpr {

// per-step outputs of the lockstep kernel (device pointers)
struct StepBuffers {
  double* obs;
  double* reward;
  uint8_t* done;
  double* era;
  double* erd;
  double* eprog;
  double* ect;
  double* est;
  int64_t* esteps;
  int64_t* eacts;
  int32_t* hh;
  int32_t* hm;
  uint32_t* status;  // per-lane cpr_episode_status bits of the current episode (always written)
};

// persistent per-lane memory of the lockstep lanes (device pointers)
struct LockBuffers {
  void* lanes;      // LockLane[n]
  double* ring;     // [RING][n] mining times of the private chain's last RING blocks
  double* spill;    // [n][cap]
  uint8_t* replay;  // [n][REPLAY_BYTES]
  // exact lanes: a lockstep lane whose episode leaves the closed form
  // (CPR_ST_LOCKSTEP_INEXACT) is simulated again on the exact event engine in Nakamoto mode
  // from its first draw and its logged actions, and continues there. alog = null: none.
  uint8_t* alog;         // [n][alog_cap] the actions taken in the lane's episode so far
  int64_t alog_cap;
  uint8_t* emem;         // [n_slots][elane_bytes] event-engine lane regions
  int64_t elane_bytes;
  void* eslots;          // eth::EthLane[n_slots]
  int32_t* efree;        // [n_slots] stack of free slots, its height at efree[n_slots]
  int32_t n_slots;
};

// per-lane bytes the fused kernel needs in HBM besides LDS
inline int64_t episode_lane_bytes(const NakParams& P) {
  return (int64_t)P.cap * 8 + REPLAY_BYTES;
}

// redo/redo_n (optional, device): flagged episodes are appended to that queue (entries
// tagged with launch_id, at most redo_cap) instead of accumulated, for launch_nak_exact_rerun
// list (optional, device, run_episodes_list_bytes): the deferred-race kernel's episodes for
// its eager second pass; null = races decided eagerly
// Where the deferred-race kernel's eager second pass runs (launch_run_episodes): on
// `stream`, after `main_done` (recorded on the launch's stream behind the main kernel), and
// `done` recorded behind it; *ran = whether a second pass was launched. Null: the second
// pass follows the main kernel on the launch's own stream.
struct SidePass {
  hipStream_t stream;
  hipEvent_t main_done, done;
  bool* ran;
};

hipError_t launch_run_episodes(const NakParams& P, uint64_t seed, uint64_t first, int64_t n_eps,
                               int32_t mode, int64_t activations, double* spill,
                               uint8_t* replay, int64_t* list, int64_t lanes,
                               cpr_episode_record* recs, cpr_summary* sum, int64_t* redo,
                               uint32_t* redo_n, uint32_t launch_id, int64_t redo_cap,
                               uint8_t* ovf, hipStream_t st, const SidePass* side = nullptr);
int64_t run_episodes_list_bytes(const NakParams& P, int32_t mode, bool recs, int64_t n_eps);
// the same fused kernel drawing from a device copy of a cpr_trace (cpr_replay)
hipError_t launch_replay_episodes(const NakParams& P, const TraceSource& src, int64_t n_eps,
                                  int32_t mode, int64_t activations, double* spill,
                                  uint8_t* replay, int64_t lanes,
                                  cpr_episode_record* recs, cpr_summary* sum, int64_t* redo,
                                  uint32_t* redo_n, uint32_t launch_id, int64_t redo_cap,
                                  uint8_t* ovf, hipStream_t st);
// EP: the batch's Ethereum lane in Nakamoto mode (observations of lanes on the exact engine)
hipError_t launch_reset(const NakParams& P, const eth::EthParams& EP, uint64_t seed,
                        const LockBuffers& B, int64_t n, const uint8_t* mask, const uint64_t* eps,
                        int unit, const double* tab_nn, const double* tab_sg, int32_t tab_n,
                        double* obs, hipStream_t st);
hipError_t launch_step(const NakParams& P, uint64_t seed, const LockBuffers& B, int64_t n,
                       const int32_t* actions, int unit, const double* tab_nn,
                       const double* tab_sg, int32_t tab_n, const StepBuffers& b,
                       hipStream_t st);
// after launch_step: lanes that left the closed form move to (or step on) the exact engine
// (EP: the batch's Ethereum lane in Nakamoto mode) and their step outputs are rewritten
hipError_t launch_lock_exact(const eth::EthParams& EP, uint64_t seed, const LockBuffers& B,
                             int64_t n, const int32_t* actions, int unit, const double* tab_nn,
                             const double* tab_sg, int32_t tab_n, const StepBuffers& b,
                             hipStream_t st);
hipError_t launch_observe_fields(const eth::EthParams& EP, const LockBuffers& B, int64_t n,
                                 int32_t* f, hipStream_t st);
hipError_t launch_policy(int32_t policy, int unit, const double* obs, int64_t n,
                         const uint8_t* table, int32_t dim, int32_t* actions, hipStream_t st);
hipError_t launch_stream_fill(uint64_t seed, uint64_t ep, uint32_t idx0, uint32_t tag, int64_t n,
                              uint32_t* out, double* exp_out, hipStream_t st);
size_t lock_lane_bytes();

// Per-node outputs of the event-engine episode kernels (cpr_node_outputs): a second
// per-lane region (activations per node, per-block reward arrays) and the [episode][node]
// output rows; mem == nullptr disables them
struct NodeOut {
  uint8_t* mem = nullptr;
  int64_t lane_bytes = 0;
  int64_t* acts = nullptr;   // [n_eps][n]
  double* rews = nullptr;    // [n_eps][n]
  int32_t* head_miner = nullptr;  // [n_eps] miner of the head block (-1 genesis / summary)
};

// Ethereum (kernels_eth.hip): mem = lanes x lane_bytes, one region per resident lane
hipError_t launch_eth_run_episodes(const eth::EthParams& P, uint64_t seed, uint64_t first,
                                   int64_t n_eps, uint8_t* mem, int64_t lane_bytes,
                                   int64_t lanes, cpr_episode_record* recs, cpr_summary* sum,
                                   hipStream_t st,
                                   const NodeOut& no = NodeOut());
hipError_t launch_eth_replay_episodes(const eth::EthParams& P, const TraceSource& src, int64_t n_eps,
                                 uint8_t* mem, int64_t lane_bytes, int64_t lanes,
                                 cpr_episode_record* recs, cpr_summary* sum, hipStream_t st,
                                   const NodeOut& no = NodeOut());
int eth_blocks_per_cu();
// event-heap nodes per lane in the LDS slab of an event-engine kernel launched with
// `blocks` workgroups (kernels_bk.hip; the B_k and Tailstorm lanes' BkMem / TsMem.hl)
int32_t ev_slab_nodes(int64_t blocks, const void* kernel);
// heap slab nodes, visibility-window vertices and dynamic LDS bytes of a B_k / Tailstorm
// kernel launched with `blocks` workgroups on n nodes (kernels_bk.hip)
struct EvSlab {
  int32_t kl, vw;
  size_t bytes;
  int32_t tw = 0;      // Tailstorm list-record window rows (TsMem.tl), 0 = none
  size_t tw_off = 0;   // its byte offset in the slab (16-aligned)
};
// lanes: used lanes per workgroup (0: all of kBlock); trec_rows: list-record window rows the
// Tailstorm fused kernel asks for (a power of 2; halved until it fits, before the heap nodes)
EvSlab ev_slab_plan(int64_t blocks, const void* kernel, int32_t n, int32_t lanes = 0,
                    int32_t trec_rows = 0);
int32_t rollout_lanes_per_wave(int64_t n, const void* kernel);
int32_t event_lanes_per_wave();
// Ethereum gym episodes on the selfish-mining network through the window lane
// (eth_window.h; ethw::win_supported): mem = lanes x ethw::win_lane_bytes; flagged episodes
// go to the exact re-run queue (redo / redo_n, entries tagged with launch_id)
hipError_t launch_eth_win_episodes(const eth::EthParams& P, uint64_t seed, uint64_t first,
                                   int64_t n_eps, uint8_t* mem, int64_t lane_bytes,
                                   int64_t lanes, cpr_episode_record* recs, cpr_summary* sum,
                                   int64_t* redo, uint32_t* redo_n, uint32_t launch_id,
                                   int64_t redo_cap, uint8_t* ovf, hipStream_t st);
int eth_win_blocks_per_cu(bool recs);
// Ethereum lockstep lanes: mem = n x lane_bytes; slots = n x eth_slot_bytes()
hipError_t launch_eth_reset(const eth::EthParams& P, uint64_t seed, uint8_t* mem,
                            int64_t lane_bytes, void* slots, int64_t n, const uint8_t* mask,
                            const uint64_t* eps, int unit, const double* tabs, int32_t tn,
                            double* obs, hipStream_t st);
hipError_t launch_eth_step(const eth::EthParams& P, uint64_t seed, uint8_t* mem,
                           int64_t lane_bytes, void* slots, int64_t n, const int32_t* actions,
                           int unit, const double* tabs, int32_t tn, const StepBuffers& b,
                           hipStream_t st);
hipError_t launch_eth_rollout(const eth::EthParams& P, uint64_t seed, uint8_t* mem,
                              int64_t lane_bytes, void* slots, int64_t n, int64_t n_steps,
                              int unit, const double* tabs, int32_t tn, double* obs,
                              double* reward, uint8_t* done, cpr_summary* sum, hipStream_t st);
hipError_t launch_eth_observe_fields(const eth::EthParams& P, uint8_t* mem, int64_t lane_bytes,
                                     const void* slots, int64_t n, int32_t* f, hipStream_t st);
hipError_t launch_eth_policy(int32_t policy, int unit, const double* obs, int64_t n,
                             const uint8_t* table, int32_t dim, int32_t* actions,
                             hipStream_t st);
size_t eth_slot_bytes();
// Exact re-runs of flagged Nakamoto episodes. Episode kernels append
// queue entries (launch << 40) | (episode index << 8) | lane status bits; one RerunLaunch
// per episode-kernel launch tells the re-run kernel where that launch's draws come from and
// where its records and summary go.
// A launcher whose translation unit lays a lane's region out larger than the region the
// library allocated refuses the launch (hipErrorInvalidValue) instead of running lanes past
// their regions. The two can only disagree in a partial rebuild: round 4's illegal memory
// access (gpurun_out/r04o_libs.log, k_bk_rollout) came from an A/B library that rebuilt
// kernels_bk.hip with a larger vote-record array (vn: 4 -> 16 bytes per slot) but linked
// the default capi.hip, which sized every lane's region by the old bk_lane_bytes
#define CPR_LAYOUT_GUARD(have, need)                  \
  do {                                                \
    if ((int64_t)(have) < (int64_t)(need)) return hipErrorInvalidValue; \
  } while (0)

// The LDS guard. hipLaunchKernelGGL does not refuse a dispatch whose static plus dynamic
// LDS exceeds the CU's 160 KiB, even after hipFuncSetAttribute refused that size: the
// queue aborts it (HSA_STATUS_ERROR_INVALID_ALLOCATION), and HIP reports the abort as "an
// illegal memory access was encountered" although no memory was accessed
// (tools/probes/lds_limit_probe.hip, profiles/r6a_lds_probe.log; the round-5 fault of the
// rejected wave-wide re-run variant). lds_dynamic_max(kernel) = the
// device's LDS per workgroup less the kernel's static LDS (hipFuncGetAttributes), cached per
// kernel and device; every launcher that asks for dynamic LDS checks its request with
// CPR_LDS_GUARD and refuses (hipErrorInvalidValue) rather than dispatch
int64_t lds_dynamic_max(const void* kernel);
#define CPR_LDS_GUARD(kernel, dyn)                                          \
  do {                                                                      \
    if ((int64_t)(dyn) > lds_dynamic_max((const void*)(kernel))) return hipErrorInvalidValue; \
  } while (0)

constexpr int64_t kRerunQueue = 1 << 22;       // queue entries per context
constexpr size_t kRerunMaxLaunches = 1 << 20;  // launches per flush (< 2^23)

struct RerunLaunch {
  eth::EthParams P;  // the Ethereum lane in Nakamoto mode, or Ethereum (window-lane episodes)
  uint64_t seed, first;
  int32_t is_trace, _pad;
  TraceSource tr;
  cpr_episode_record* recs;
  cpr_summary* sum;
  int64_t lane_bytes;
  // overflow flags [n_eps] (zeroed at registration): a flagged episode that found the
  // queue full writes 0x80 | its status bits here instead (k_rerun_overflow re-runs it)
  uint8_t* ovf;
  int64_t n_eps;
  // Nakamoto episodes of the closed-form lane re-run as hybrids (nak_hybrid.h): its
  // parameters (cap: spill slots for a whole episode) and 1 when the launcher's condition
  // holds; the lane region then ends with hybrid_bytes(NP.cap) for the closed form
  NakParams NP;
  int32_t hybrid, _pad2;
};

// all queued re-runs (count on the device) in one launch of `lanes` one-wave workgroups,
// each with a lane region of lane_bytes at mem + i x lane_bytes; lds_bytes (the largest
// eth_rest_bytes of the launches, capped at 160 KiB) puts all but the block ring in LDS;
// then, only if the queue overflowed (count > queue_cap), the overflow flags of every
// launch (k_rerun_overflow on the same lane regions)
hipError_t launch_nak_exact_rerun(const RerunLaunch* launches, int64_t n_launches,
                                  const int64_t* queue, const uint32_t* queue_n,
                                  int64_t queue_cap, uint8_t* mem, int64_t lane_bytes,
                                  int64_t lds_bytes, int64_t lanes, hipStream_t st);

// B_k (kernels_bk.hip): mem = lanes x lane_bytes; lockstep slots = n x bk_slot_bytes()
hipError_t launch_bk_run_episodes(const bk::BkParams& P, uint64_t seed, uint64_t first,
                                  int64_t n_eps, uint8_t* mem, int64_t lane_bytes, int64_t lanes,
                                  cpr_episode_record* recs, cpr_summary* sum, hipStream_t st,
                                   const NodeOut& no = NodeOut());
hipError_t launch_bk_replay_episodes(const bk::BkParams& P, const TraceSource& src, int64_t n_eps,
                                 uint8_t* mem, int64_t lane_bytes, int64_t lanes,
                                 cpr_episode_record* recs, cpr_summary* sum, hipStream_t st,
                                   const NodeOut& no = NodeOut());
hipError_t launch_bk_reset(const bk::BkParams& P, uint64_t seed, uint8_t* mem, int64_t lane_bytes,
                           void* slots, int64_t n, const uint8_t* mask, const uint64_t* eps,
                           int unit, const double* tabs, int32_t tn, double* obs, hipStream_t st);
hipError_t launch_bk_step(const bk::BkParams& P, uint64_t seed, uint8_t* mem, int64_t lane_bytes,
                          void* slots, int64_t n, const int32_t* actions, int unit,
                          const double* tabs, int32_t tn, const StepBuffers& b, hipStream_t st);
hipError_t launch_bk_rollout(const bk::BkParams& P, uint64_t seed, uint8_t* mem,
                             int64_t lane_bytes, void* slots, int64_t n, int64_t n_steps,
                             int unit, const double* tabs, int32_t tn, double* obs,
                             double* reward, uint8_t* done, cpr_summary* sum, hipStream_t st);
hipError_t launch_bk_observe_fields(const bk::BkParams& P, uint8_t* mem, int64_t lane_bytes,
                                    const void* slots, int64_t n, int32_t* f, hipStream_t st);
hipError_t launch_bk_policy(const bk::BkParams& P, int unit, const double* obs, int64_t n,
                            int32_t* actions, hipStream_t st);
size_t bk_slot_bytes();
int bk_blocks_per_cu();

// Tailstorm (kernels_ts.hip), same shapes as the B_k launchers
hipError_t launch_ts_run_episodes(const ts::TsParams& P, uint64_t seed, uint64_t first,
                                  int64_t n_eps, uint8_t* mem, int64_t lane_bytes, int64_t lanes,
                                  cpr_episode_record* recs, cpr_summary* sum, hipStream_t st,
                                   const NodeOut& no = NodeOut());
hipError_t launch_ts_replay_episodes(const ts::TsParams& P, const TraceSource& src, int64_t n_eps,
                                 uint8_t* mem, int64_t lane_bytes, int64_t lanes,
                                 cpr_episode_record* recs, cpr_summary* sum, hipStream_t st,
                                   const NodeOut& no = NodeOut());
hipError_t launch_ts_reset(const ts::TsParams& P, uint64_t seed, uint8_t* mem, int64_t lane_bytes,
                           void* slots, int64_t n, const uint8_t* mask, const uint64_t* eps,
                           int unit, const double* tabs, int32_t tn, double* obs, hipStream_t st);
hipError_t launch_ts_step(const ts::TsParams& P, uint64_t seed, uint8_t* mem, int64_t lane_bytes,
                          void* slots, int64_t n, const int32_t* actions, int unit,
                          const double* tabs, int32_t tn, const StepBuffers& b, hipStream_t st);
hipError_t launch_ts_rollout(const ts::TsParams& P, uint64_t seed, uint8_t* mem,
                             int64_t lane_bytes, void* slots, int64_t n, int64_t n_steps,
                             int unit, const double* tabs, int32_t tn, double* obs,
                             double* reward, uint8_t* done, cpr_summary* sum, hipStream_t st);
hipError_t launch_ts_observe_fields(const ts::TsParams& P, uint8_t* mem, int64_t lane_bytes,
                                    const void* slots, int64_t n, int32_t* f, hipStream_t st);
hipError_t launch_ts_policy(int32_t policy, int32_t k, int unit, const double* obs, int64_t n,
                            const uint8_t* table, int32_t dim, int32_t* actions,
                            hipStream_t st);
size_t ts_slot_bytes();
int ts_blocks_per_cu();
// resident 256-lane workgroups per CU of the k_run_episodes instantiation a launch of this
// configuration runs (recs: per-episode records asked for)
int run_episodes_blocks_per_cu(const NakParams& P, int32_t mode, bool recs);

// FC'16 abstract-model episodes (fc16_lane.h), lanes = multiple of kBlock
hipError_t launch_fc16_episodes(const fc16::Fc16Params& P, uint64_t seed, uint64_t first,
                                int64_t n_eps, int64_t lanes, cpr_episode_record* recs,
                                cpr_summary* sum, hipStream_t st);

}  // namespace cpr

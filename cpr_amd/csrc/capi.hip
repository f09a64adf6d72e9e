// libcpr_hip C ABI (include/cpr_hip.h): host side. Validation mirrors the reference's
// engine.ml:37-51 (Parameters.t) and network.ml:61-76 (selfish_mining) so invalid
// configurations fail with the same messages; all episode work runs on the device.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <memory>
#include <string>
#include <deque>
#include <vector>

#include "../../include/cpr_hip.h"
#include "eth_window.h"
#include "kernels.h"
#include "nak_hybrid.h"

using namespace cpr;

#ifndef CPR_VERSION_STRING
#define CPR_VERSION_STRING "cpr-hip 0.1.0 (gfx950)"
#endif

static thread_local std::string g_err;

static int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define HIP_TRY(expr)                                                                    \
  do {                                                                                   \
    hipError_t e_ = (expr);                                                              \
    if (e_ != hipSuccess)                                                                \
      return fail(CPR_E_HIP, std::string(#expr " failed: ") + hipGetErrorString(e_));   \
  } while (0)

// device allocation owned by one object (freed on destruction, so every early return of
// an entry point releases its scratch buffers); not copyable
struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
  DevBuf() = default;
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  ~DevBuf() { release(); }
  hipError_t ensure(size_t n) {
    if (n <= bytes) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
    hipError_t e = hipMalloc(&p, n);
    if (e == hipSuccess) bytes = n;
    return e;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
  }
};

struct cpr_ctx {
  int device;
  hipStream_t stream;
  int cus;
  // Nakamoto episodes flagged by the closed-form lane wait here for their exact re-run
  // (k_nak_exact_rerun), which runs at the next synchronization point, all of them in one
  // launch: rq = [kRerunQueue] int64 entries + a uint32 counter; one RerunLaunch per
  // episode-kernel launch since then
  DevBuf rq, rtab, rmem;
  // cpr_rerun_stats: per flush, HIP events around the re-run kernels and the count of
  // episodes the launches since the previous flush queued (copied to pinned host memory
  // before the counter is cleared; e2 follows that copy). Every flush folds the records
  // whose e2 has completed into rr_* and recycles them (drain_flush_recs), and waits for the
  // oldest when kFlushRecMax are outstanding, so a context that never asks for the stats
  // holds a bounded set of events and pinned words
  struct FlushRec {
    hipEvent_t e0 = nullptr, e1 = nullptr, e2 = nullptr;
    uint32_t* cnt = nullptr;  // pinned host word
  };
  std::deque<FlushRec> fl_pending;
  std::vector<FlushRec> fl_free;
  int64_t rr_episodes = 0, rr_flushes = 0;
  double rr_ms = 0.0;
  std::vector<RerunLaunch> rlaunch, rlaunch_up;
  // entries a launch may append (kRerunQueue; CPR_RERUN_QUEUE_CAP lowers it for tests);
  // an episode that finds the queue full waits in its launch's overflow flags: one byte
  // per episode of every launch since the last flush, carved from the chunks of `ovf` in
  // order (chunk ovf_chunk, ovf_used bytes taken). Chunks are never reallocated, so
  // filling one forces no flush until kOvfMaxChunks are in use (1 GiB of flags, ~200
  // launches of the bench's 5.2M episodes): a flush costs the latency of one exact episode
  // (~80 ms at the gym's 2016 steps), paid once per synchronization
  int64_t rq_cap = kRerunQueue;
  std::vector<std::unique_ptr<DevBuf>> ovf;
  size_t ovf_chunk = 0, ovf_used = 0;
  // per-lane scratch regions of fused-episode launches (event-engine rings and heaps, the
  // Nakamoto lane's spill / time log / tie-replay scratch), shared by every batch of the
  // context: launches on the context's stream run in order, so one grow-only pool serves an
  // alpha x gamma sweep of any number of batches
  DevBuf pool;
  // work-queue counter of the event-engine fused-episode launches (wave_sched.h
  // ev_next_episode), zeroed on the stream before each launch
  DevBuf wq;
  // the deferred-race kernels' eager second passes (kernels.hip launch_run_episodes) run on
  // `side`, behind their launch's main kernel, so that they overlap the next launch on
  // `stream`. Each reads one of two list buffers; list_ev[i] marks the end of the pass that
  // reads lists[i], and the next launch that writes lists[i] waits for it on `stream`.
  // side_join makes `stream` wait for every pass still pending (before a flush, a
  // synchronization, or any read of summaries and the re-run queue)
  hipStream_t side = nullptr;
  hipEvent_t main_ev = nullptr;
  DevBuf lists[2];
  hipEvent_t list_ev[2] = {nullptr, nullptr};
  bool list_pending[2] = {false, false};
  int list_i = 0;
};

static hipError_t side_join(cpr_ctx* c) {
  for (int i = 0; i < 2; ++i)
    if (c->list_pending[i]) {
      const hipError_t e = hipStreamWaitEvent(c->stream, c->list_ev[i], 0);
      if (e != hipSuccess) return e;
      c->list_pending[i] = false;
    }
  return hipSuccess;
}

// the context's scratch pool with at least `bytes`
static hipError_t ctx_pool(cpr_ctx* c, size_t bytes, void** out) {
  hipError_t e = c->pool.ensure(bytes);
  *out = c->pool.p;
  return e;
}

// a zeroed work-queue counter for the next event-engine launch on the context's stream
// (launches on the stream run in order, so one counter serves them all)
static hipError_t ctx_next(cpr_ctx* c, unsigned long long** out) {
  hipError_t e = c->wq.ensure(8);
  if (e == hipSuccess) e = hipMemsetAsync(c->wq.p, 0, 8, c->stream);
  *out = (unsigned long long*)c->wq.p;
  return e;
}

static size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

struct cpr_batch {
  cpr_ctx* ctx;
  cpr_config cfg;
  NakParams P;
  eth::EthParams EP;     // CPR_PROTO_ETHEREUM
  bool is_eth = false;   // Ethereum lockstep lanes share bk_lmem / bk_slots
  bool nak_ev = false;   // Nakamoto on the event engine (nak_on_event_engine): Ethereum lanes
                         // in Nakamoto mode (EP)
  int64_t eth_bytes = 0;
  bk::BkParams BP;       // CPR_PROTO_BK
  DevBuf bk_lmem, bk_slots;  // lockstep lanes: n_lanes x bk_bytes, n_lanes slots
  int64_t bk_bytes = 0;
  ts::TsParams TP;       // CPR_PROTO_TAILSTORM (shares bk_lmem / bk_slots)
  fc16::Fc16Params FP;   // CPR_PROTO_FC16
  bool is_ev = false;    // B_k or Tailstorm event-engine lanes
  // Nakamoto fused episodes: exact re-runs of flagged episodes on the event engine
  bool has_rerun = false;
  eth::EthParams NEP;    // the Ethereum lane in Nakamoto mode
  int64_t nak_bytes = 0;
  bool async_launch = false;  // last launch came from cpr_run_episodes_async
  std::vector<uint8_t> table_host;
  DevBuf table_dev, tabs_dev;  // policy table; unit-observation tables
  DevBuf summary, records;
  DevBuf pol_obs, pol_act;  // cpr_policy_actions staging, reused across calls
  DevBuf tr_off, tr_miner, tr_delay, tr_pow, tr_key, tr_ldelay;  // cpr_replay trace copy
  // lockstep lanes
  DevBuf lanes, lring, lspill, lreplay, l_obs, l_act, l_rew, l_done, l_mask, l_eps, l_info;
  // exact Nakamoto lockstep lanes (LockBuffers): action log, event-engine slots
  DevBuf l_alog, l_emem, l_eslots, l_efree;
  int64_t alog_cap = 0;
  int32_t n_exact_slots = 0;
  bool reset_done = false;
  int32_t tab_n = 4096;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  double last_ms = 0.0;
  int64_t last_acts = 0;
  int64_t last_lanes = 0, last_resident = 0;  // cpr_launch_shape
};

extern "C" {

const char* cpr_version(void) { return CPR_VERSION_STRING; }
int cpr_abi_version(void) { return CPR_ABI_VERSION; }
const char* cpr_last_error(void) { return g_err.c_str(); }

int cpr_device_count(int* out) {
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess) return fail(CPR_E_HIP, std::string("hipGetDeviceCount: ") + hipGetErrorString(e));
  *out = n;
  return CPR_OK;
}

static int flush_reruns(cpr_ctx* c);

int cpr_ctx_create(int device, cpr_ctx** out) {
  if (!out) return fail(CPR_E_INVALID_ARG, "out is NULL");
  int n = 0;
  HIP_TRY(hipGetDeviceCount(&n));
  if (device < 0 || device >= n) return fail(CPR_E_INVALID_ARG, "no such HIP device");
  HIP_TRY(hipSetDevice(device));
  hipDeviceProp_t prop;
  HIP_TRY(hipGetDeviceProperties(&prop, device));
  cpr_ctx* c = new cpr_ctx;
  c->device = device;
  c->cus = prop.multiProcessorCount;
  hipError_t e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->side, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&c->main_ev, hipEventDisableTiming);
  for (int i = 0; i < 2 && e == hipSuccess; ++i)
    e = hipEventCreateWithFlags(&c->list_ev[i], hipEventDisableTiming);
  if (e != hipSuccess) {
    delete c;
    return fail(CPR_E_HIP, std::string("hipStreamCreate: ") + hipGetErrorString(e));
  }
  *out = c;
  return CPR_OK;
}

int cpr_ctx_destroy(cpr_ctx* c) {
  if (!c) return CPR_OK;
  (void)hipSetDevice(c->device);
  // pending work first: queued exact re-runs complete their callers' summaries and records
  (void)flush_reruns(c);  // joins the side stream's second passes first
  (void)hipStreamSynchronize(c->stream);
  (void)hipStreamSynchronize(c->side);
  c->fl_free.insert(c->fl_free.end(), c->fl_pending.begin(), c->fl_pending.end());
  c->fl_pending.clear();
  for (cpr_ctx::FlushRec& r : c->fl_free) {
    (void)hipEventDestroy(r.e0);
    (void)hipEventDestroy(r.e1);
    (void)hipEventDestroy(r.e2);
    (void)hipHostFree(r.cnt);
  }
  (void)hipStreamDestroy(c->stream);
  (void)hipStreamDestroy(c->side);
  (void)hipEventDestroy(c->main_ev);
  for (int i = 0; i < 2; ++i) {
    (void)hipEventDestroy(c->list_ev[i]);
    c->lists[i].release();
  }
  c->rq.release();
  c->rtab.release();
  c->rmem.release();
  c->wq.release();
  delete c;
  return CPR_OK;
}

int cpr_synchronize(cpr_ctx* c) {
  HIP_TRY(hipSetDevice(c->device));
  int rc = flush_reruns(c);  // joins the side stream first
  if (rc) return rc;
  HIP_TRY(hipStreamSynchronize(c->stream));
  return CPR_OK;
}

static uint64_t alpha_threshold(double alpha) {
  double t = alpha * 4294967296.0;
  if (t <= 0.0) return 0;
  if (t >= 4294967296.0) return 4294967296ull;
  return (uint64_t)t;
}

// engine.ml:37-51 and network.ml:61-76 (messages kept verbatim)
static int validate_eth(const cpr_config* c, eth::EthParams* P);

// the keyed miner draw for compute weights 1..n (models.ml:3-28), as the oracle's
// weight_thresholds: thr[i] = floor(sum_{j<=i} w_j / sum w * 2^32), i < n - 1
static void clique_thresholds(int n, uint32_t* thr) {
  double total = 0.0, cum = 0.0;
  for (int i = 0; i < n; ++i) total += (double)(i + 1);
  for (int i = 0; i + 1 < n; ++i) {
    cum += (double)(i + 1);
    const double t = cum / total * 4294967296.0;
    thr[i] = t <= 0.0 ? 0u : (t >= 4294967295.0 ? 4294967295u : (uint32_t)t);
  }
}

static int validate_bk(const cpr_config* c, bk::BkParams* P);
static int validate_ts(const cpr_config* c, ts::TsParams* P);

// Nakamoto configurations the closed-form lane does not cover run on the event engine:
// honest cliques; Simulator.loop tasks on the selfish-mining network at gamma = 0 (messages
// at t = +inf, drained after the last activation); and loop tasks whose message delays make
// overlapping windows common (the withholding sweep's 1e-4 defender delay overlaps about
// once per 10,000 activations, models.ml:54), which the closed-form lane would hand to
// the same engine episode by episode anyway
// the random attacker of the reference's policy tests (cpr_protocols.ml:658-782) decides in
// its handler: Simulator.loop tasks (the gym's agent takes actions from its caller)
static const char* random_policy_msg =
    "random attacker actions: Simulator.loop tasks (CPR_MODE_LOOP) on the event engines";

static bool nak_on_event_engine(const cpr_config* c) {
  if (c->protocol != CPR_PROTO_NAKAMOTO) return false;
  if (c->network == CPR_NET_HONEST_CLIQUE || c->network == CPR_NET_EXP_CLIQUE) return true;
  if (c->network != CPR_NET_SELFISH_MINING || c->mode != CPR_MODE_LOOP) return false;
  if (c->gamma == 0.0) return true;
  const double prop = c->propagation_delay > 0 ? c->propagation_delay : 1e-9;
  const double dd = (double)c->defenders;
  const double span = std::max(prop, (dd - 1.) / dd * prop / c->gamma);
  return !(span * (double)c->activations < 1e-3 * c->activation_delay);
}

// FC'16 abstract model (fc16.rs:141-158 FC16SSZwPT::new: Bernoulli(alpha), Bernoulli(gamma),
// Bernoulli(1 / horizon) reject probabilities outside [0, 1])
static int validate_fc16(const cpr_config* c, fc16::Fc16Params* P) {
  if (std::isnan(c->alpha) || c->alpha < 0. || c->alpha > 1.)
    return fail(CPR_E_INVALID_ARG, "alpha < 0 || alpha > 1");
  if (std::isnan(c->gamma) || c->gamma < 0. || c->gamma > 1.)
    return fail(CPR_E_INVALID_ARG, "gamma < 0 || gamma > 1");
  if (!(c->horizon >= 1.)) return fail(CPR_E_INVALID_ARG, "horizon must be >= 1");
  if (c->mode != CPR_MODE_GYM) return fail(CPR_E_UNSUPPORTED, "FC16 runs gym episodes");
  if (c->policy < CPR_FC16_POLICY_HONEST || c->policy > CPR_FC16_POLICY_TABLE)
    return fail(CPR_E_INVALID_ARG, "unknown policy");
  memset(P, 0, sizeof(*P));
  if (c->policy == CPR_FC16_POLICY_TABLE) {
    const int64_t D = c->policy_table_dim;
    if (!c->policy_table || D <= 0 || D > 256)
      return fail(CPR_E_INVALID_ARG, "policy table missing or dim out of range (1..256)");
    for (int64_t i = 0; i < D * D * 3; i++)
      if (c->policy_table[i] > 3) return fail(CPR_E_INVALID_ARG, "policy table action out of range");
    P->table_dim = (int32_t)D;
  }
  P->t_alpha = alpha_threshold(c->alpha);
  P->t_gamma = alpha_threshold(c->gamma);
  P->t_term = alpha_threshold(1.0 / c->horizon);
  P->max_steps = c->max_steps > 0 ? c->max_steps : (int64_t)1 << 30;
  P->policy = c->policy;
  return CPR_OK;
}

static int validate(const cpr_config* c, NakParams* P, eth::EthParams* EP, bk::BkParams* BP,
                    ts::TsParams* TP) {
  if (c->protocol == CPR_PROTO_ETHEREUM) return validate_eth(c, EP);
  if (c->protocol == CPR_PROTO_BK) return validate_bk(c, BP);
  if (c->protocol == CPR_PROTO_TAILSTORM) return validate_ts(c, TP);
  if (c->protocol != CPR_PROTO_NAKAMOTO)
    return fail(CPR_E_UNSUPPORTED, "protocol not implemented on the device yet");
  if (c->network == CPR_NET_HONEST_CLIQUE) {
    // every node honest: the event engine in Nakamoto mode (no closed form for cliques)
    cpr_config c2 = *c;
    c2.protocol = CPR_PROTO_ETHEREUM;
    c2.policy = CPR_ETH_POLICY_HONEST;
    c2.reward_scheme = CPR_REWARD_CONSTANT;
    const int rc = validate_eth(&c2, EP);
    if (rc) return rc;
    EP->nak = 1;
    return CPR_OK;
  }
  if (std::isnan(c->activation_delay)) return fail(CPR_E_INVALID_ARG, "activation_delay cannot be NaN");
  if (std::isnan(c->alpha)) return fail(CPR_E_INVALID_ARG, "alpha cannot be NaN");
  if (std::isnan(c->gamma)) return fail(CPR_E_INVALID_ARG, "gamma cannot be NaN");
  if (c->alpha < 0. || c->alpha > 1.) return fail(CPR_E_INVALID_ARG, "alpha < 0 || alpha > 1");
  if (c->gamma < 0. || c->gamma > 1.) return fail(CPR_E_INVALID_ARG, "gamma < 0 || gamma > 1");
  if (c->activation_delay <= 0.) return fail(CPR_E_INVALID_ARG, "activation_delay <= 0");
  if (c->mode != CPR_MODE_GYM && c->mode != CPR_MODE_LOOP)
    return fail(CPR_E_INVALID_ARG, "unknown mode");
  if (c->policy < CPR_POLICY_HONEST || c->policy > CPR_POLICY_RANDOM)
    return fail(CPR_E_INVALID_ARG, "unknown policy");
  if (c->policy == CPR_POLICY_RANDOM && !(c->mode == CPR_MODE_LOOP && nak_on_event_engine(c)))
    return fail(CPR_E_UNSUPPORTED, random_policy_msg);
  if (c->policy == CPR_POLICY_TABLE) {
    if (!c->policy_table || c->policy_table_dim <= 0 || c->policy_table_dim > 256)
      return fail(CPR_E_INVALID_ARG, "policy table missing or dim out of range (1..256)");
    for (int i = 0; i < c->policy_table_dim * c->policy_table_dim * 2; i++)
      if (c->policy_table[i] > 3) return fail(CPR_E_INVALID_ARG, "policy table action out of range");
  }
  if (nak_on_event_engine(c)) {
    // Simulator.loop on the selfish-mining network at gamma = 0: the attacker's messages
    // arrive at t = +inf and the loop drains them after the last activation
    // (simulator.ml:519-533); no closed form, so the event engine in Nakamoto mode runs it
    cpr_config c2 = *c;
    c2.protocol = CPR_PROTO_ETHEREUM;
    c2.policy = CPR_ETH_POLICY_HONEST;
    c2.reward_scheme = CPR_REWARD_CONSTANT;
    const int rc = validate_eth(&c2, EP);
    if (rc) return rc;
    EP->nak = 1;
    EP->policy = c->policy;
    EP->table_dim = c->policy_table_dim;
    return CPR_OK;
  }
  memset(P, 0, sizeof(*P));
  P->ev = c->activation_delay;
  P->t_att = alpha_threshold(c->alpha);
  P->policy = c->policy;
  P->table_dim = c->policy_table_dim;
  if (c->network == CPR_NET_SELFISH_MINING) {
    if (c->defenders < 1) return fail(CPR_E_INVALID_ARG, "defenders < 0");
    if (c->defenders < 2) return fail(CPR_E_INVALID_ARG, "defenders must be at least 2");
    if (c->defenders > 64)
      return fail(CPR_E_UNSUPPORTED, "device lanes support at most 64 defenders");
    const double dd = (double)c->defenders;
    if (c->gamma > (dd - 1.) / dd)
      return fail(CPR_E_INVALID_ARG, "gamma must not be greater ( (defenders - 1) / defenders )");
    const double prop = c->propagation_delay > 0 ? c->propagation_delay : 1e-9;
    P->d = c->defenders;
    P->delta = prop;
    P->dmax = (dd - 1.) / dd * prop / c->gamma;
    P->arrive = std::isfinite(P->dmax) ? 1 : 0;
  } else if (c->network == CPR_NET_TWO_AGENTS) {
    if (c->mode == CPR_MODE_GYM)
      return fail(CPR_E_UNSUPPORTED, "the gym engine always uses the selfish-mining network");
    P->d = 1;
    P->delta = 0.0;
    P->dmax = 0.0;
    P->arrive = 1;
  } else if (c->network == CPR_NET_ABSTRACT_GAMMA) {
    // flagged abstract-gamma mode (include/cpr_hip.h): zero delays, coin-decided races
    if (c->mode != CPR_MODE_GYM)
      return fail(CPR_E_UNSUPPORTED, "the abstract-gamma mode runs gym episodes");
    if (c->defenders < 1 || c->defenders > 64)
      return fail(CPR_E_INVALID_ARG, "abstract gamma: 1..64 defenders");
    P->d = c->defenders;
    P->delta = 0.0;
    P->dmax = 0.0;
    P->arrive = 1;
    P->abstract_g = 1;
    P->gamma = c->gamma;
  } else {
    return fail(CPR_E_INVALID_ARG, "unknown network");
  }
  int64_t span;  // activations per episode + 1 (bound on chain length and clock index)
  if (c->mode == CPR_MODE_GYM) {
    const int64_t ms = c->max_steps > 0 ? c->max_steps : INT64_MAX;
    P->max_steps = ms;
    P->max_progress = c->max_progress > 0 ? c->max_progress : __builtin_inf();
    P->max_time = c->max_time > 0 ? c->max_time : __builtin_inf();
    span = ms < (1 << 20) ? ms + 2 : 4096;
  } else {
    if (c->activations <= 0) return fail(CPR_E_INVALID_ARG, "activations <= 0");
    if (c->activations > (1 << 24)) return fail(CPR_E_UNSUPPORTED, "activations > 2^24");
    P->max_steps = INT64_MAX;
    P->max_progress = __builtin_inf();
    P->max_time = __builtin_inf();
    span = c->activations + 2;
  }
  P->cap = (int32_t)(((std::min<int64_t>(span, 1 << 20) + 63) / 64) * 64);
  return CPR_OK;
}

// Ethereum: engine.ml:37-51 checks shared with Nakamoto, network.ml:61-76, ethereum_ssz
// policies 0..4, Constant / Discount rewards
static int validate_eth(const cpr_config* c, eth::EthParams* P) {
  if (std::isnan(c->activation_delay)) return fail(CPR_E_INVALID_ARG, "activation_delay cannot be NaN");
  if (std::isnan(c->alpha)) return fail(CPR_E_INVALID_ARG, "alpha cannot be NaN");
  if (std::isnan(c->gamma)) return fail(CPR_E_INVALID_ARG, "gamma cannot be NaN");
  if (c->alpha < 0. || c->alpha > 1.) return fail(CPR_E_INVALID_ARG, "alpha < 0 || alpha > 1");
  if (c->gamma < 0. || c->gamma > 1.) return fail(CPR_E_INVALID_ARG, "gamma < 0 || gamma > 1");
  if (c->activation_delay <= 0.) return fail(CPR_E_INVALID_ARG, "activation_delay <= 0");
  if (c->mode != CPR_MODE_GYM && c->mode != CPR_MODE_LOOP)
    return fail(CPR_E_INVALID_ARG, "unknown mode");
  if (c->policy < CPR_ETH_POLICY_HONEST || c->policy > CPR_ETH_POLICY_RANDOM)
    return fail(CPR_E_INVALID_ARG, "unknown policy");
  if (c->policy == CPR_ETH_POLICY_RANDOM && c->mode != CPR_MODE_LOOP)
    return fail(CPR_E_UNSUPPORTED, random_policy_msg);
  if (c->reward_scheme != CPR_REWARD_CONSTANT && c->reward_scheme != CPR_REWARD_DISCOUNT)
    return fail(CPR_E_INVALID_ARG, "unknown incentive scheme");
  if (c->policy == CPR_ETH_POLICY_TABLE) {
    const int64_t D = c->policy_table_dim;
    if (!c->policy_table || D <= 0 || D > 64)
      return fail(CPR_E_INVALID_ARG, "policy table missing or dim out of range (1..64)");
    for (int64_t i = 0; i < D * D * 2; i++)
      if (c->policy_table[i] > 23) return fail(CPR_E_INVALID_ARG, "policy table action out of range");
  }
  memset(P, 0, sizeof(*P));
  P->table_dim = c->policy == CPR_ETH_POLICY_TABLE ? c->policy_table_dim : 0;
  P->ev = c->activation_delay;
  P->t_att = alpha_threshold(c->alpha);
  P->policy = c->policy;
  P->scheme = c->reward_scheme;
  P->mode = c->mode;
  if (c->network == CPR_NET_SELFISH_MINING) {
    if (c->defenders < 1) return fail(CPR_E_INVALID_ARG, "defenders < 0");
    if (c->defenders < 2) return fail(CPR_E_INVALID_ARG, "defenders must be at least 2");
    if (c->defenders > 64)
      return fail(CPR_E_UNSUPPORTED, "device lanes support at most 64 defenders");
    const double dd = (double)c->defenders;
    if (c->gamma > (dd - 1.) / dd)
      return fail(CPR_E_INVALID_ARG, "gamma must not be greater ( (defenders - 1) / defenders )");
    const double prop = c->propagation_delay > 0 ? c->propagation_delay : 1e-9;
    P->d = c->defenders;
    P->net = 0;
    P->delta = prop;
    P->dmax = (dd - 1.) / dd * prop / c->gamma;
  } else if (c->network == CPR_NET_TWO_AGENTS) {
    if (c->mode == CPR_MODE_GYM)
      return fail(CPR_E_UNSUPPORTED, "the gym engine always uses the selfish-mining network");
    P->d = 1;
    P->net = 1;
  } else if (c->network == CPR_NET_HONEST_CLIQUE) {
    // models.ml:3-28: n honest nodes with compute i + 1, uniform link delays
    if (c->mode != CPR_MODE_LOOP)
      return fail(CPR_E_UNSUPPORTED, "honest cliques run Simulator.loop tasks (CPR_MODE_LOOP)");
    if (c->defenders < 2 || c->defenders > 64)
      return fail(CPR_E_INVALID_ARG, "honest clique: 2..64 nodes (cfg.defenders)");
    const bool dflt = std::isnan(c->delay_lo) && std::isnan(c->delay_hi);  // NaN: models.ml default
    const double lo = dflt ? 0.5 : c->delay_lo, hi = dflt ? 1.5 : c->delay_hi;
    if (!(lo >= 0.) || !(hi >= lo)) return fail(CPR_E_INVALID_ARG, "delay_lo/delay_hi");
    P->d = c->defenders - 1;
    P->net = 2;
    P->lo = lo;
    P->hi = hi;
    clique_thresholds(c->defenders, P->thr);
  } else if (c->network == CPR_NET_EXP_CLIQUE) {
    // cpr_protocols.ml:478-485: symmetric clique, exponential link delays, node 0 runs the
    // attack policy (ethereum_ssz, or nakamoto_ssz in Nakamoto mode); keyed equal-weight
    // miner draw (attacker threshold 1/n)
    if (c->mode != CPR_MODE_LOOP)
      return fail(CPR_E_UNSUPPORTED, "the gym engine always uses the selfish-mining network");
    if (c->defenders < 1 || c->defenders > 63)
      return fail(CPR_E_INVALID_ARG, "exponential clique: 1..63 defenders");
    if (!(c->propagation_delay > 0.) || !std::isfinite(c->propagation_delay))
      return fail(CPR_E_INVALID_ARG, "exponential clique: propagation_delay must be positive");
    P->d = c->defenders;
    P->net = 3;
    P->delta = c->propagation_delay;
    P->t_att = alpha_threshold(1.0 / (double)(c->defenders + 1));
  } else {
    return fail(CPR_E_INVALID_ARG, "unknown network");
  }
  P->n = P->d + 1;
  int64_t span;
  if (c->mode == CPR_MODE_GYM) {
    const int64_t ms = c->max_steps > 0 ? c->max_steps : INT64_MAX;
    P->max_steps = ms;
    P->max_progress = c->max_progress > 0 ? c->max_progress : __builtin_inf();
    P->max_time = c->max_time > 0 ? c->max_time : __builtin_inf();
    span = ms < (1 << 20) ? ms + 2 : 4096;
  } else {
    if (c->activations <= 0) return fail(CPR_E_INVALID_ARG, "activations <= 0");
    if (c->activations > (1 << 24)) return fail(CPR_E_UNSUPPORTED, "activations > 2^24");
    P->max_steps = INT64_MAX;
    P->activations = c->activations;
    P->max_progress = __builtin_inf();
    P->max_time = __builtin_inf();
    span = c->activations + 2;
  }
  // the block ring holds a whole episode up to 2^15 blocks (longer episodes flag
  // CPR_ST_CAPACITY only if a fork outlives the ring); heap: 512 in-flight events per node
  int32_t cb = 64;
  while (cb < span && cb < (1 << 15)) cb <<= 1;
  P->cap_b = cb;
  // gamma = 0: messages at t = +inf stay in the skew heap (they shape its tie order);
  // otherwise an attacker release shares every withheld block at once, d messages each
  // (a 300-block release at alpha .45, gamma .9 overflowed 512 events per node), and each
  // block is released at most once: d messages per block of the episode bound the heap
  int64_t extra = 0;
  const int64_t ext = P->mode == CPR_MODE_LOOP ? span : std::min<int64_t>(span, 8192);
  if (P->net == 0 && !std::isfinite(P->dmax))
    extra = 2 * (int64_t)P->d * ext;
  else if (P->net == 0 || P->net == 3)
    extra = (int64_t)P->d * ext;
  P->cap_e = 64 + 512 * P->n + (int32_t)std::min<int64_t>(extra, 1 << 24);
  return CPR_OK;
}

// vertex-ring window of the B_k / Tailstorm lanes (see validate_bk)
static constexpr int32_t kRingWindow = 4096;
// HBM budget for the per-lane regions of the event-engine lanes (288 GB per MI355X)
static constexpr int64_t kLaneBudget = 96ll << 30;

// B_k: engine.ml:37-51 checks shared with Nakamoto, network.ml:61-76, bk.ml k >= 1,
// Constant / Block rewards, bk_ssz policies 0..3 or a table
static int validate_bk(const cpr_config* c, bk::BkParams* P) {
  if (std::isnan(c->activation_delay)) return fail(CPR_E_INVALID_ARG, "activation_delay cannot be NaN");
  if (std::isnan(c->alpha)) return fail(CPR_E_INVALID_ARG, "alpha cannot be NaN");
  if (std::isnan(c->gamma)) return fail(CPR_E_INVALID_ARG, "gamma cannot be NaN");
  if (c->alpha < 0. || c->alpha > 1.) return fail(CPR_E_INVALID_ARG, "alpha < 0 || alpha > 1");
  if (c->gamma < 0. || c->gamma > 1.) return fail(CPR_E_INVALID_ARG, "gamma < 0 || gamma > 1");
  if (c->activation_delay <= 0.) return fail(CPR_E_INVALID_ARG, "activation_delay <= 0");
  if (c->mode != CPR_MODE_GYM && c->mode != CPR_MODE_LOOP)
    return fail(CPR_E_INVALID_ARG, "unknown mode");
  if (c->k < 1) return fail(CPR_E_INVALID_ARG, "k must be positive");
  if (c->k > 64) return fail(CPR_E_UNSUPPORTED, "device lanes support k <= 64");
  if (c->reward_scheme != CPR_REWARD_CONSTANT && c->reward_scheme != CPR_REWARD_BLOCK)
    return fail(CPR_E_INVALID_ARG, "'" + std::to_string(c->reward_scheme) +
                                       "' is not a valid parameter choice, try 'block' or 'constant'");
  if (c->policy < CPR_BK_POLICY_HONEST || c->policy > CPR_BK_POLICY_RANDOM)
    return fail(CPR_E_INVALID_ARG, "unknown policy");
  if (c->policy == CPR_BK_POLICY_RANDOM && c->mode != CPR_MODE_LOOP)
    return fail(CPR_E_UNSUPPORTED, random_policy_msg);
  memset(P, 0, sizeof(*P));
  if (c->policy == CPR_BK_POLICY_TABLE) {
    const int64_t D = c->policy_table_dim;
    if (!c->policy_table || D <= 0 || D > 64)
      return fail(CPR_E_INVALID_ARG, "policy table missing or dim out of range (1..64)");
    const int64_t sz = D * D * (c->k + 1) * (c->k + 1) * 3;
    for (int64_t i = 0; i < sz; i++)
      if (c->policy_table[i] > 7) return fail(CPR_E_INVALID_ARG, "policy table action out of range");
    P->table_dim = (int32_t)D;
  }
  P->ev = c->activation_delay;
  P->t_att = alpha_threshold(c->alpha);
  P->policy = c->policy;
  P->scheme = c->reward_scheme;
  P->mode = c->mode;
  P->k = c->k;
  if (c->network == CPR_NET_SELFISH_MINING) {
    if (c->defenders < 1) return fail(CPR_E_INVALID_ARG, "defenders < 0");
    if (c->defenders < 2) return fail(CPR_E_INVALID_ARG, "defenders must be at least 2");
    if (c->defenders > 64)
      return fail(CPR_E_UNSUPPORTED, "device lanes support at most 64 defenders");
    const double dd = (double)c->defenders;
    if (c->gamma > (dd - 1.) / dd)
      return fail(CPR_E_INVALID_ARG, "gamma must not be greater ( (defenders - 1) / defenders )");
    const double prop = c->propagation_delay > 0 ? c->propagation_delay : 1e-9;
    P->d = c->defenders;
    P->net = 0;
    P->delta = prop;
    P->dmax = (dd - 1.) / dd * prop / c->gamma;
  } else if (c->network == CPR_NET_TWO_AGENTS) {
    if (c->mode == CPR_MODE_GYM)
      return fail(CPR_E_UNSUPPORTED, "the gym engine always uses the selfish-mining network");
    P->d = 1;
    P->net = 1;
  } else if (c->network == CPR_NET_HONEST_CLIQUE) {
    // models.ml:3-28: n honest nodes with compute i + 1, uniform link delays; node 0 runs
    // the honest protocol too (the policy is ignored)
    if (c->mode != CPR_MODE_LOOP)
      return fail(CPR_E_UNSUPPORTED, "honest cliques run Simulator.loop tasks (CPR_MODE_LOOP)");
    if (c->defenders < 2 || c->defenders > 64)
      return fail(CPR_E_INVALID_ARG, "honest clique: 2..64 nodes (cfg.defenders)");
    const bool dflt = std::isnan(c->delay_lo) && std::isnan(c->delay_hi);  // NaN: models.ml default
    const double lo = dflt ? 0.5 : c->delay_lo, hi = dflt ? 1.5 : c->delay_hi;
    if (!(lo >= 0.) || !(hi >= lo)) return fail(CPR_E_INVALID_ARG, "delay_lo/delay_hi");
    P->d = c->defenders - 1;
    P->net = 2;
    P->lo = lo;
    P->hi = hi;
    clique_thresholds(c->defenders, P->thr);
  } else if (c->network == CPR_NET_EXP_CLIQUE) {
    // cpr_protocols.ml:478-485: symmetric clique, exponential link delays, node 0 runs the
    // attack policy; the oracle's keyed draw for equal compute 1/n (attacker threshold)
    if (c->mode != CPR_MODE_LOOP)
      return fail(CPR_E_UNSUPPORTED, "the gym engine always uses the selfish-mining network");
    if (c->defenders < 1 || c->defenders > 63)
      return fail(CPR_E_INVALID_ARG, "exponential clique: 1..63 defenders");
    if (!(c->propagation_delay > 0.) || !std::isfinite(c->propagation_delay))
      return fail(CPR_E_INVALID_ARG, "exponential clique: propagation_delay must be positive");
    P->d = c->defenders;
    P->net = 3;
    P->delta = c->propagation_delay;
    P->t_att = alpha_threshold(1.0 / (double)(c->defenders + 1));
  } else {
    return fail(CPR_E_INVALID_ARG, "unknown network");
  }
  P->n = P->d + 1;
  int64_t span;
  if (c->mode == CPR_MODE_GYM) {
    const int64_t ms = c->max_steps > 0 ? c->max_steps : INT64_MAX;
    P->max_steps = ms;
    P->max_progress = c->max_progress > 0 ? c->max_progress : __builtin_inf();
    P->max_time = c->max_time > 0 ? c->max_time : __builtin_inf();
    span = ms < (1 << 20) ? ms + 2 : 8192;
  } else {
    if (c->activations <= 0) return fail(CPR_E_INVALID_ARG, "activations <= 0");
    if (c->activations > (1 << 24)) return fail(CPR_E_UNSUPPORTED, "activations > 2^24");
    P->max_steps = INT64_MAX;
    P->activations = c->activations;
    P->max_progress = __builtin_inf();
    P->max_time = __builtin_inf();
    span = c->activations * 2 + 2;  // votes + blocks
  }
  // vertex ring: a window of at most 4096 vertices (a whole 2048-step gym episode); longer
  // runs flag CPR_ST_CAPACITY only if something older than the window is read (a fork
  // that outlives it). Small per-lane regions let the grid reach resident capacity.
  int32_t cv = 64;
  while (cv < span + 64 && cv < kRingWindow) cv <<= 1;
  P->cap_v = cv;
  P->cap_q = cv / 2;
  P->cap_d = 64;
  P->cap_e = 256 + 512 * P->n +
             (std::isfinite(P->dmax) || P->net == 1
                  ? 0
                  : (int32_t)(2 * P->d * std::min<int64_t>(span, 8192)));
  return CPR_OK;
}

// Tailstorm: engine.ml:37-51 checks, network.ml:61-76, tailstorm.ml k >= 1, the four
// incentive schemes and three sub-block selections, tailstorm_ssz policies 0..6
static int validate_ts(const cpr_config* c, ts::TsParams* P) {
  // the B_k checks cover everything but the scheme, selection and policy ranges
  cpr_config cb = *c;
  cb.protocol = CPR_PROTO_BK;
  cb.reward_scheme = CPR_REWARD_CONSTANT;
  cb.policy = CPR_BK_POLICY_HONEST;
  bk::BkParams B;
  int rc = validate_bk(&cb, &B);
  if (rc) return rc;
  if (c->reward_scheme != CPR_REWARD_CONSTANT && c->reward_scheme != CPR_REWARD_DISCOUNT &&
      c->reward_scheme != CPR_REWARD_PUNISH && c->reward_scheme != CPR_REWARD_HYBRID)
    return fail(CPR_E_INVALID_ARG, "'" + std::to_string(c->reward_scheme) +
                                       "' is not a valid parameter choice, try 'constant', "
                                       "'discount', 'punish' or 'hybrid'");
  if (c->subblock_selection < CPR_SELECT_ALTRUISTIC || c->subblock_selection > CPR_SELECT_OPTIMAL)
    return fail(CPR_E_INVALID_ARG, "'" + std::to_string(c->subblock_selection) +
                                       "' is not a valid parameter choice, try 'altruistic', "
                                       "'heuristic' or 'optimal'");
  if (c->policy < CPR_TS_POLICY_HONEST || c->policy > CPR_TS_POLICY_RANDOM)
    return fail(CPR_E_INVALID_ARG, "unknown policy");
  if (c->policy == CPR_TS_POLICY_RANDOM && c->mode != CPR_MODE_LOOP)
    return fail(CPR_E_UNSUPPORTED, random_policy_msg);
  if (c->policy == CPR_TS_POLICY_TABLE) {
    const int64_t D = c->policy_table_dim;
    if (!c->policy_table || D <= 0 || D > 64)
      return fail(CPR_E_INVALID_ARG, "policy table missing or dim out of range (1..64)");
    const int64_t sz = D * D * (c->k + 1) * (c->k + 1) * 3;
    for (int64_t i = 0; i < sz; i++)
      if (c->policy_table[i] > 7) return fail(CPR_E_INVALID_ARG, "policy table action out of range");
  }
  memset(P, 0, sizeof(*P));
  P->opt_budget = ts::TS_OPT_BUDGET;
  P->table_dim = c->policy == CPR_TS_POLICY_TABLE ? c->policy_table_dim : 0;
  P->t_att = B.t_att;
  P->d = B.d;
  P->n = B.n;
  P->net = B.net;
  P->mode = B.mode;
  P->policy = c->policy;
  P->scheme = c->reward_scheme;
  P->selection = c->subblock_selection;
  P->k = c->k;
  P->ev = B.ev;
  P->delta = B.delta;
  P->dmax = B.dmax;
  P->max_steps = B.max_steps;
  P->activations = B.activations;
  P->max_progress = B.max_progress;
  P->max_time = B.max_time;
  P->lo = B.lo;
  P->hi = B.hi;
  memcpy(P->thr, B.thr, sizeof(P->thr));
  // gym: one vertex per attacker interaction plus summaries; loop: ~ (1 + 1/k) per
  // activation. Vertex ring covers the whole episode up to 2^16 vertices.
  const int64_t span = c->mode == CPR_MODE_GYM
                           ? (B.max_steps < (1 << 20) ? B.max_steps + 2 : 8192)
                           : c->activations * 2 + 2;
  int32_t cv = 64;
  while (cv < span + 64 && cv < kRingWindow) cv <<= 1;
  P->cap_v = cv;
  P->cap_q = cv / 2;
  P->cap_d = 64;
  P->cap_e = 256 + 512 * P->n +
             (std::isfinite(P->dmax) || P->net == 1
                  ? 0
                  : (int32_t)(2 * P->d * std::min<int64_t>(span, 8192)));
  return CPR_OK;
}

int cpr_batch_create(cpr_ctx* ctx, const cpr_config* cfg, cpr_batch** out) {
  if (!ctx || !cfg || !out) return fail(CPR_E_INVALID_ARG, "NULL argument");
  NakParams P;
  eth::EthParams EP;
  bk::BkParams BP;
  ts::TsParams TP;
  memset(&P, 0, sizeof(P));
  memset(&EP, 0, sizeof(EP));
  memset(&BP, 0, sizeof(BP));
  memset(&TP, 0, sizeof(TP));
  fc16::Fc16Params FP;
  memset(&FP, 0, sizeof(FP));
  int rc = cfg->protocol == CPR_PROTO_FC16 ? validate_fc16(cfg, &FP)
                                           : validate(cfg, &P, &EP, &BP, &TP);
  if (rc) return rc;
  HIP_TRY(hipSetDevice(ctx->device));
  cpr_batch* b = new cpr_batch;
  b->ctx = ctx;
  b->cfg = *cfg;
  b->P = P;
  b->EP = EP;
  b->BP = BP;
  b->TP = TP;
  b->FP = FP;
  b->eth_bytes = eth::eth_lane_bytes(EP.cap_b, EP.cap_e, EP.n);
  if (cfg->protocol == CPR_PROTO_BK) b->bk_bytes = bk::bk_lane_bytes(BP);
  if (cfg->protocol == CPR_PROTO_TAILSTORM) b->bk_bytes = ts::ts_lane_bytes(TP);
  b->is_ev = cfg->protocol == CPR_PROTO_BK || cfg->protocol == CPR_PROTO_TAILSTORM;
  b->is_eth = cfg->protocol == CPR_PROTO_ETHEREUM;
  b->nak_ev = nak_on_event_engine(cfg);
  b->cfg.policy_table = nullptr;
  if (cfg->protocol == CPR_PROTO_BK && cfg->policy == CPR_BK_POLICY_TABLE) {
    const size_t D = (size_t)cfg->policy_table_dim, K1 = (size_t)cfg->k + 1;
    b->table_host.assign(cfg->policy_table, cfg->policy_table + D * D * K1 * K1 * 3);
  } else if ((cfg->protocol == CPR_PROTO_NAKAMOTO && cfg->policy == CPR_POLICY_TABLE) ||
             (cfg->protocol == CPR_PROTO_ETHEREUM && cfg->policy == CPR_ETH_POLICY_TABLE)) {
    const size_t nb = (size_t)cfg->policy_table_dim * cfg->policy_table_dim * 2;
    b->table_host.assign(cfg->policy_table, cfg->policy_table + nb);
  } else if (cfg->protocol == CPR_PROTO_FC16 && cfg->policy == CPR_FC16_POLICY_TABLE) {
    const size_t D = (size_t)cfg->policy_table_dim;
    b->table_host.assign(cfg->policy_table, cfg->policy_table + D * D * 3);
  } else if (cfg->protocol == CPR_PROTO_TAILSTORM && cfg->policy == CPR_TS_POLICY_TABLE) {
    const size_t D = (size_t)cfg->policy_table_dim, K1 = (size_t)cfg->k + 1;
    b->table_host.assign(cfg->policy_table, cfg->policy_table + D * D * K1 * K1 * 3);
  }
  // unit-observation tables (ssz_tools.ml:36-39) evaluated with the host libm:
  // [2/pi atan(i) | 0.5 + atan(i - N)/pi (2N) | 2/pi atan(i/k)], i < N
  const double kscale =
      (cfg->protocol == CPR_PROTO_BK || cfg->protocol == CPR_PROTO_TAILSTORM) ? (double)cfg->k : 1.0;
  std::vector<double> tabs(4 * (size_t)b->tab_n);
  for (int i = 0; i < b->tab_n; i++) tabs[i] = 2. / M_PI * std::atan((double)i / 1.0);
  for (int i = 0; i < 2 * b->tab_n; i++)
    tabs[b->tab_n + i] = 0.5 + (1. / M_PI * std::atan((double)(i - b->tab_n) / 1.0));
  for (int i = 0; i < b->tab_n; i++)
    tabs[3 * b->tab_n + i] = 2. / M_PI * std::atan((double)i / kscale);
  hipError_t e = b->tabs_dev.ensure(tabs.size() * sizeof(double));
  if (e == hipSuccess)
    e = hipMemcpy(b->tabs_dev.p, tabs.data(), tabs.size() * sizeof(double), hipMemcpyHostToDevice);
  if (e == hipSuccess && !b->table_host.empty()) {
    e = b->table_dev.ensure(b->table_host.size());
    if (e == hipSuccess)
      e = hipMemcpy(b->table_dev.p, b->table_host.data(), b->table_host.size(),
                    hipMemcpyHostToDevice);
  }
  if (e != hipSuccess) {
    delete b;
    return fail(CPR_E_HIP, std::string("batch buffers: ") + hipGetErrorString(e));
  }
  b->P.table = (const uint8_t*)b->table_dev.p;
  b->BP.table = (const uint8_t*)b->table_dev.p;
  b->EP.table = (const uint8_t*)b->table_dev.p;  // Nakamoto-mode or ethereum_ssz table
  b->TP.table = (const uint8_t*)b->table_dev.p;
  b->FP.table = (const uint8_t*)b->table_dev.p;
  if (cfg->protocol == CPR_PROTO_NAKAMOTO && !b->nak_ev) {
    // the same episode on the exact event engine: Ethereum lane, no uncles, nakamoto_ssz
    // policy (validated above); configurations it cannot hold keep the lane's flags
    cpr_config c2 = *cfg;
    c2.protocol = CPR_PROTO_ETHEREUM;
    c2.policy = CPR_ETH_POLICY_HONEST;
    c2.reward_scheme = CPR_REWARD_CONSTANT;
    const std::string keep_err = g_err;
    if (validate_eth(&c2, &b->NEP) == CPR_OK) {
      b->NEP.nak = 1;
      b->NEP.policy = cfg->policy;
      b->NEP.table = b->P.table;
      b->NEP.table_dim = cfg->policy_table_dim;
      b->nak_bytes = eth::eth_lane_bytes(b->NEP.cap_b, b->NEP.cap_e, b->NEP.n);
      b->has_rerun = true;
    }
    g_err = keep_err;
  }
  *out = b;
  return CPR_OK;
}

// lanes the device holds at once for this batch's fused-episode kernel (before any launch)
static int64_t batch_resident(cpr_batch* b) {
  const int64_t cus = b->ctx->cus;
  if (b->cfg.protocol == CPR_PROTO_FC16) return cus * 8 * 256;
  if (b->cfg.protocol == CPR_PROTO_ETHEREUM || b->nak_ev) return cus * eth_blocks_per_cu() * 256;
  if (b->is_ev)
    return cus * (b->cfg.protocol == CPR_PROTO_TAILSTORM ? ts_blocks_per_cu() : bk_blocks_per_cu()) *
           256;
  return cus * run_episodes_blocks_per_cu(b->P, b->cfg.mode, false) * 256;
}

int cpr_launch_shape(cpr_batch* b, int64_t* lanes, int64_t* resident) {
  if (!b) return fail(CPR_E_INVALID_ARG, "NULL argument");
  HIP_TRY(hipSetDevice(b->ctx->device));
  if (lanes) *lanes = b->last_lanes;
  if (resident) *resident = b->last_lanes ? b->last_resident : batch_resident(b);
  return CPR_OK;
}

int cpr_rerun_hbm_retries(cpr_ctx* c, int64_t* retries) {
  if (!c || !retries) return fail(CPR_E_INVALID_ARG, "NULL argument");
  *retries = 0;
  if (!c->rq.p) return CPR_OK;
  HIP_TRY(hipSetDevice(c->device));
  HIP_TRY(side_join(c));
  uint32_t v = 0;
  HIP_TRY(hipStreamSynchronize(c->stream));
  HIP_TRY(hipMemcpy(&v, (char*)c->rq.p + (size_t)kRerunQueue * 8 + 4, 4, hipMemcpyDeviceToHost));
  *retries = v;
  return CPR_OK;
}

// fold finished flush records (oldest first: one stream, so they finish in order) into the
// totals and recycle them; wait: every one (cpr_rerun_stats), else only those done, plus the
// oldest while more than kFlushRecMax are outstanding
constexpr size_t kFlushRecMax = 32;

static int drain_flush_recs(cpr_ctx* c, bool wait) {
  while (!c->fl_pending.empty()) {
    const cpr_ctx::FlushRec r = c->fl_pending.front();
    if (wait || c->fl_pending.size() > kFlushRecMax) {
      HIP_TRY(hipEventSynchronize(r.e2));
    } else {
      const hipError_t q = hipEventQuery(r.e2);
      if (q == hipErrorNotReady) break;
      HIP_TRY(q);
    }
    float t = 0.f;
    HIP_TRY(hipEventElapsedTime(&t, r.e0, r.e1));
    c->rr_ms += t;
    c->rr_episodes += *r.cnt;
    c->rr_flushes += 1;
    c->fl_free.push_back(r);
    c->fl_pending.pop_front();
  }
  return CPR_OK;
}

int cpr_rerun_stats(cpr_ctx* c, int64_t* episodes, int64_t* flushes, double* ms) {
  if (!c) return fail(CPR_E_INVALID_ARG, "NULL argument");
  HIP_TRY(hipSetDevice(c->device));
  if (const int rc = drain_flush_recs(c, true)) return rc;
  if (episodes) *episodes = c->rr_episodes;
  if (flushes) *flushes = c->rr_flushes;
  if (ms) *ms = c->rr_ms;
  return CPR_OK;
}

int cpr_lockstep_coverage(cpr_batch* b, int64_t* log_steps, int64_t* exact_slots) {
  if (!b) return fail(CPR_E_INVALID_ARG, "NULL argument");
  if (log_steps) *log_steps = b->l_alog.p ? b->alog_cap : 0;
  if (exact_slots) *exact_slots = b->l_alog.p ? b->n_exact_slots : 0;
  return CPR_OK;
}

int cpr_last_launch(cpr_batch* b, double* kernel_ms, int64_t* activations) {
  if (!b) return fail(CPR_E_INVALID_ARG, "NULL argument");
  if (b->async_launch) {  // cpr_run_episodes_async: the caller has synchronized
    float ms = 0.f;
    HIP_TRY(hipEventElapsedTime(&ms, b->ev0, b->ev1));
    b->last_ms = ms;
    b->last_acts = -1;  // not known without reading the caller's device summary
    b->async_launch = false;
  }
  if (kernel_ms) *kernel_ms = b->last_ms;
  if (activations) *activations = b->last_acts;
  return CPR_OK;
}

int cpr_batch_destroy(cpr_batch* b) {
  if (!b) return CPR_OK;
  (void)hipSetDevice(b->ctx->device);
  (void)hipStreamSynchronize(b->ctx->stream);
  (void)flush_reruns(b->ctx);  // pending re-runs may read this batch's buffers
  (void)hipStreamSynchronize(b->ctx->stream);
  if (b->ev0) (void)hipEventDestroy(b->ev0);
  if (b->ev1) (void)hipEventDestroy(b->ev1);
  b->bk_lmem.release();
  b->bk_slots.release();
  for (DevBuf* d : {&b->table_dev, &b->tabs_dev, &b->summary,
                    &b->records, &b->lanes, &b->lring, &b->lspill, &b->lreplay,
                    &b->l_obs, &b->l_act, &b->l_rew, &b->l_done, &b->l_mask, &b->l_eps,
                    &b->l_info, &b->l_alog, &b->l_emem, &b->l_eslots, &b->l_efree, &b->tr_off, &b->tr_miner, &b->tr_delay, &b->tr_pow,
                    &b->tr_key, &b->tr_ldelay})
    d->release();
  delete b;
  return CPR_OK;
}

// lanes per launch: exactly the resident capacity (occupancy API: workgroups per CU at
// this kernel's register/LDS use x CUs x 256), bounded by a 16 GiB budget for per-lane HBM
// exact Nakamoto re-runs: one-wave workgroups of the re-run kernel
constexpr int64_t kRerunLanes = 512;
constexpr int64_t kRerunLanesMax = 8192;  // one workgroup per queued episode, up to this

static int64_t episode_lanes(cpr_batch* b, int64_t n_eps, bool recs) {
  const int64_t full =
      (int64_t)b->ctx->cus * run_episodes_blocks_per_cu(b->P, b->cfg.mode, recs) * 256;
  const int64_t budget = (int64_t)(16ll << 30) / episode_lane_bytes(b->P);
  int64_t lanes = std::min(full, std::max<int64_t>(256, budget));
  // A/B: a share of the resident grid (percent), e.g. for launches that run concurrently
  if (const char* v = getenv("CPR_GRID_SCALE")) {
    const int64_t pc = atoll(v);
    if (pc > 0 && pc < 100) lanes = lanes * pc / 100;
  }
  lanes = std::max<int64_t>(256, (lanes / 256) * 256);
  // equal rounds: the episodes of a launch spread evenly over the fewest rounds of the
  // resident grid, so the last round is not a partly empty one (every lane's episode has
  // the same trip count in the gym)
  const int64_t rounds = std::max<int64_t>(1, (n_eps + lanes - 1) / lanes);
  const int64_t even = ((n_eps + rounds - 1) / rounds + 255) / 256 * 256;
  return std::max<int64_t>(256, std::min(lanes, even));
}

// Re-run every queued flagged Nakamoto episode of the launches since the last flush, in
// one k_nak_exact_rerun launch on the context's stream (after those launches, before the
// caller reads summaries or records), then empty the queue.
constexpr size_t kOvfMaxChunks = 4;  // overflow-flag chunks (256 MiB each) before a flush

static int flush_reruns(cpr_ctx* c) {
  // the side stream's second passes append to the queue and add to summaries: everything
  // after this point on the stream (the re-runs, the caller's reads) comes after them
  HIP_TRY(side_join(c));
  if (c->rlaunch.empty()) return CPR_OK;
  int64_t lb = 0, rest = 0;
  for (const RerunLaunch& r : c->rlaunch) {
    // the re-run region's layout (rerun_episode): the engine lane, then a hybrid's
    // closed-form ring, spill and tie-replay scratch (hybrid_mem); a launch registered with
    // a smaller region is refused here rather than run past it
    const int64_t need = eth::eth_lane_bytes(r.P.cap_b, r.P.cap_e, r.P.n) +
                         (r.hybrid ? hybrid_bytes(r.NP.cap) : 0);
    if (r.lane_bytes < need || (r.hybrid && r.NP.cap < r.P.max_steps + 2))
      return fail(CPR_E_HIP, "re-run region smaller than its layout (" +
                                 std::to_string(r.lane_bytes) + " < " + std::to_string(need) +
                                 " bytes)");
    lb = std::max(lb, r.lane_bytes);
    rest = std::max(rest, eth::eth_rest_bytes(r.P.cap_b, r.P.cap_e, r.P.n));
  }
  c->rlaunch_up.swap(c->rlaunch);  // keeps the host table alive for the async copy
  c->rlaunch.clear();
  const size_t tb = c->rlaunch_up.size() * sizeof(RerunLaunch);
  HIP_TRY(c->rtab.ensure(tb));
  HIP_TRY(hipMemcpyAsync(c->rtab.p, c->rlaunch_up.data(), tb, hipMemcpyHostToDevice, c->stream));
  uint32_t* qn = (uint32_t*)((char*)c->rq.p + (size_t)kRerunQueue * 8);
  // how many episodes the launches queued (a flush is a synchronization point anyway). Up to
  // one per CU: one-wave workgroups of 512 with the lane's heap, visibility and scratch in up
  // to a whole CU's LDS, the fastest per episode (a re-run is one dependent chain). More
  // (the headline's sweep queues ~140 per step, ~2,850 in a 20-step timed region, half of
  // them gamma = 0 re-runs whose +inf messages keep the heap large): LDS of that size would
  // run them one CU at a time, round after round, so each episode gets a workgroup of its own
  // with its region in HBM instead and they all run at once
  int64_t lanes = kRerunLanes, lds_rest = rest;
#ifndef CPR_FLUSH_ADAPTIVE
#define CPR_FLUSH_ADAPTIVE 1
#endif
  if (CPR_FLUSH_ADAPTIVE) {
    HIP_TRY(hipStreamSynchronize(c->stream));
    uint32_t nq = 0;
    HIP_TRY(hipMemcpy(&nq, qn, sizeof(nq), hipMemcpyDeviceToHost));
    if ((int64_t)nq > (int64_t)c->cus) {
      lanes = std::min<int64_t>((int64_t)nq, kRerunLanesMax);
      lds_rest = 0;
      // A/B: LDS per workgroup in this mode (the heap at the capacity that fits, an episode
      // that outgrows it again in HBM); 0 = the whole region in HBM
      if (const char* v = getenv("CPR_RERUN_WIDE_LDS")) lds_rest = std::min<int64_t>(rest, atoll(v));
    }
  }
  if (c->rmem.ensure((size_t)lanes * (size_t)lb) != hipSuccess) {
    // the wide grid's regions do not fit: the default grid (its LDS mode), episodes looping
    // over its workgroups, rather than failing the caller's synchronization
    (void)hipGetLastError();
    lanes = kRerunLanes;
    lds_rest = rest;
    HIP_TRY(c->rmem.ensure((size_t)lanes * (size_t)lb));
  }
  if (const int rc = drain_flush_recs(c, false)) return rc;
  cpr_ctx::FlushRec fr;
  if (!c->fl_free.empty()) {
    fr = c->fl_free.back();
    c->fl_free.pop_back();
  } else {
    HIP_TRY(hipEventCreate(&fr.e0));
    HIP_TRY(hipEventCreate(&fr.e1));
    HIP_TRY(hipEventCreate(&fr.e2));
    HIP_TRY(hipHostMalloc((void**)&fr.cnt, sizeof(uint32_t)));
  }
  HIP_TRY(hipEventRecord(fr.e0, c->stream));
  HIP_TRY(launch_nak_exact_rerun((const RerunLaunch*)c->rtab.p, (int64_t)c->rlaunch_up.size(),
                                 (const int64_t*)c->rq.p, qn, c->rq_cap, (uint8_t*)c->rmem.p,
                                 lb, lds_rest, lanes, c->stream));
  HIP_TRY(hipEventRecord(fr.e1, c->stream));
  HIP_TRY(hipMemcpyAsync(fr.cnt, qn, sizeof(uint32_t), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipEventRecord(fr.e2, c->stream));
  c->fl_pending.push_back(fr);
  HIP_TRY(hipMemsetAsync(qn, 0, 4, c->stream));
  c->ovf_chunk = 0;  // the next launches' flags follow these re-runs on the stream
  c->ovf_used = 0;
  return CPR_OK;
}

// A launch whose flagged episodes the exact event engine re-runs at the next
// synchronization point (flush_reruns): its parameters (EP: the Ethereum lane, in Nakamoto
// mode for the closed-form Nakamoto lane), stream and outputs join the context's table;
// the kernel appends (launch_id << 40) | (episode << 8) | flags to the queue
static int register_rerun(cpr_batch* b, const eth::EthParams& EP, int64_t lane_bytes,
                          uint64_t first, const TraceSource* tr, cpr_episode_record* rec_dev,
                          cpr_summary* sum_dev, int64_t n_eps, int64_t** redo,
                          uint32_t** redo_n, uint32_t* launch_id, uint8_t** ovf,
                          const NakParams* hybrid = nullptr) {
  cpr_ctx* c = b->ctx;
  const size_t need = align256((size_t)std::max<int64_t>(1, n_eps));
  // tests force a small queue (CPR_RERUN_QUEUE_CAP) to exercise the overflow flags; a new
  // capacity takes effect at a flush (all launches of one flush share it)
  int64_t cap = kRerunQueue;
  if (const char* v = getenv("CPR_RERUN_QUEUE_CAP"))
    cap = std::max<int64_t>(0, std::min<int64_t>(kRerunQueue, atoll(v)));
  if (cap != c->rq_cap) {
    int rc = flush_reruns(c);
    if (rc) return rc;
    c->rq_cap = cap;
  }
  if (c->rlaunch.size() >= kRerunMaxLaunches) {
    int rc = flush_reruns(c);
    if (rc) return rc;
  }
  // the launch's flags: the rest of the current chunk, else the next chunk that holds them
  // (a new one if none does; earlier chunks stay, queued kernels may still read them).
  // Chunks are reused from the first after every flush; once kOvfMaxChunks are taken the
  // launches so far are flushed first, so many large asynchronous launches between two
  // synchronizations do not keep adding chunks for the life of the context
  for (int pass = 0;; ++pass) {
    while (c->ovf_chunk < c->ovf.size() && c->ovf_used + need > c->ovf[c->ovf_chunk]->bytes) {
      ++c->ovf_chunk;
      c->ovf_used = 0;
    }
    if (c->ovf_chunk < c->ovf.size() || c->ovf.size() < kOvfMaxChunks || pass > 0) break;
    const int rc = flush_reruns(c);  // resets ovf_chunk / ovf_used to chunk 0
    if (rc) return rc;
  }
  if (c->ovf_chunk == c->ovf.size()) {
    c->ovf.emplace_back(new DevBuf());
    HIP_TRY(c->ovf.back()->ensure(std::max(need, (size_t)256 << 20)));
  }
  *ovf = (uint8_t*)c->ovf[c->ovf_chunk]->p + c->ovf_used;
  HIP_TRY(hipMemsetAsync(*ovf, 0, need, c->stream));
  c->ovf_used += need;
  if (!c->rq.p) {
    HIP_TRY(c->rq.ensure((size_t)kRerunQueue * 8 + 64));
    // launch counter and the cumulative HBM-retry counter (cpr_rerun_hbm_retries)
    HIP_TRY(hipMemsetAsync((char*)c->rq.p + (size_t)kRerunQueue * 8, 0, 8, c->stream));
  }
  RerunLaunch rl;
  memset(&rl, 0, sizeof(rl));
  rl.P = EP;
  rl.P.next = nullptr;
  rl.seed = b->cfg.seed;
  rl.first = first;
  rl.is_trace = tr ? 1 : 0;
  if (tr) rl.tr = *tr;
  rl.recs = rec_dev;
  rl.sum = sum_dev;
  rl.lane_bytes = lane_bytes;
  rl.ovf = *ovf;
  rl.n_eps = n_eps;
  if (hybrid) {  // nak_hybrid.h: the closed form's state after the engine's region
    rl.NP = *hybrid;
    rl.hybrid = 1;
    rl.lane_bytes = lane_bytes + hybrid_bytes(hybrid->cap);
  }
  *launch_id = (uint32_t)c->rlaunch.size();
  c->rlaunch.push_back(rl);
  *redo = (int64_t*)c->rq.p;
  *redo_n = (uint32_t*)((char*)c->rq.p + (size_t)kRerunQueue * 8);
  return CPR_OK;
}

// The window lane (eth_window.h) takes Ethereum gym episodes on the selfish-mining network
// whose whole episode fits its block ring: the ring does not wrap (WinLane::append fails
// instead), so an episode of max_steps + 1 activations (+ genesis) must fit cap_b, or every
// episode would end in W_REDO and a one-lane exact re-run. max_progress / max_time only end
// episodes earlier (each lane leaves its loop on its own done). CPR_ETH_WINDOW=0 sends them
// to the event engine instead (A/B runs)
static bool eth_window_ok(const cpr_batch* b) {
  const char* v = getenv("CPR_ETH_WINDOW");
  return (v == nullptr || atoi(v) != 0) && ethw::win_supported(b->EP) &&
         b->EP.max_steps <= (int64_t)b->EP.cap_b - 2;
}

static int run_async_ethwin(cpr_batch* b, int64_t n, uint64_t first, cpr_summary* sum_dev,
                            cpr_episode_record* rec_dev) {
  const int64_t wbytes = ethw::win_lane_bytes(b->EP.cap_b);
  const int64_t full = (int64_t)b->ctx->cus * eth_win_blocks_per_cu(rec_dev != nullptr) * 256;
  const int64_t budget = kLaneBudget / wbytes;
  int64_t lanes = std::min(full, std::max<int64_t>(256, budget));
  lanes = std::max<int64_t>(256, (lanes / 256) * 256);
  // equal rounds of the resident grid (every episode has the same trip count)
  const int64_t rounds = std::max<int64_t>(1, (n + lanes - 1) / lanes);
  lanes = std::max<int64_t>(256, std::min(lanes, ((n + rounds - 1) / rounds + 255) / 256 * 256));
  b->last_lanes = lanes;
  b->last_resident = full;
  void* mem = nullptr;
  HIP_TRY(ctx_pool(b->ctx, (size_t)lanes * (size_t)wbytes, &mem));
  if (!b->ev0) {
    HIP_TRY(hipEventCreate(&b->ev0));
    HIP_TRY(hipEventCreate(&b->ev1));
  }
  int64_t* redo = nullptr;
  uint32_t* redo_n = nullptr;
  uint32_t launch_id = 0;
  uint8_t* ovf = nullptr;
  const int rc = register_rerun(b, b->EP, b->eth_bytes, first, nullptr, rec_dev, sum_dev, n,
                                &redo, &redo_n, &launch_id, &ovf);
  if (rc) return rc;
  // episodes beyond the first round from the context's work queue (a lane that finishes
  // early takes the next); CPR_NAK_WQ=0 keeps the static grid stride (A/B)
  eth::EthParams EP = b->EP;
  const char* wq = getenv("CPR_NAK_WQ");
  if (!(wq && wq[0] == '0')) HIP_TRY(ctx_next(b->ctx, &EP.next));
  HIP_TRY(hipEventRecord(b->ev0, b->ctx->stream));
  HIP_TRY(launch_eth_win_episodes(EP, b->cfg.seed, first, n, (uint8_t*)mem, wbytes, lanes,
                                  rec_dev, sum_dev, redo, redo_n, launch_id, b->ctx->rq_cap,
                                  ovf, b->ctx->stream));
  HIP_TRY(hipEventRecord(b->ev1, b->ctx->stream));
  return CPR_OK;
}

// Ethereum lanes: resident capacity bounded by kLaneBudget for the per-lane regions
static int run_async_eth(cpr_batch* b, int64_t n, uint64_t first, const TraceSource* tr,
                         cpr_summary* sum_dev, cpr_episode_record* rec_dev) {
  if (!tr && !b->nak_ev && eth_window_ok(b)) return run_async_ethwin(b, n, first, sum_dev, rec_dev);
  const int64_t full = (int64_t)b->ctx->cus * eth_blocks_per_cu() * 256;
  const int64_t budget = kLaneBudget / b->eth_bytes;
  int64_t lanes = std::min(full, std::max<int64_t>(256, budget));
  lanes = std::min(lanes, ((n + 255) / 256) * 256);
  lanes = std::max<int64_t>(256, (lanes / 256) * 256);
  b->last_lanes = lanes;
  b->last_resident = full;
  void* mem = nullptr;
  HIP_TRY(ctx_pool(b->ctx, (size_t)lanes * (size_t)b->eth_bytes, &mem));
  if (!b->ev0) {
    HIP_TRY(hipEventCreate(&b->ev0));
    HIP_TRY(hipEventCreate(&b->ev1));
  }
  eth::EthParams EP = b->EP;
  HIP_TRY(ctx_next(b->ctx, &EP.next));
  HIP_TRY(hipEventRecord(b->ev0, b->ctx->stream));
  if (tr)
    HIP_TRY(launch_eth_replay_episodes(EP, *tr, n, (uint8_t*)mem, b->eth_bytes,
                                       lanes, rec_dev, sum_dev, b->ctx->stream));
  else
    HIP_TRY(launch_eth_run_episodes(EP, b->cfg.seed, first, n, (uint8_t*)mem,
                                    b->eth_bytes, lanes, rec_dev, sum_dev, b->ctx->stream));
  HIP_TRY(hipEventRecord(b->ev1, b->ctx->stream));
  return CPR_OK;
}

// B_k / Tailstorm lanes: resident capacity bounded by kLaneBudget for the per-lane regions
static int run_async_bk(cpr_batch* b, int64_t n, uint64_t first, const TraceSource* tr,
                        cpr_summary* sum_dev, cpr_episode_record* rec_dev) {
  const bool tsp = b->cfg.protocol == CPR_PROTO_TAILSTORM;
  const int64_t full = (int64_t)b->ctx->cus * (tsp ? ts_blocks_per_cu() : bk_blocks_per_cu()) * 256;
  const int64_t budget = kLaneBudget / b->bk_bytes;
  int64_t lanes = std::min(full, std::max<int64_t>(256, budget));
  lanes = std::min(lanes, ((n + 255) / 256) * 256);
  lanes = std::max<int64_t>(256, (lanes / 256) * 256);
  b->last_lanes = lanes;
  b->last_resident = full;
  void* pool = nullptr;
  HIP_TRY(ctx_pool(b->ctx, (size_t)lanes * (size_t)b->bk_bytes, &pool));
  if (!b->ev0) {
    HIP_TRY(hipEventCreate(&b->ev0));
    HIP_TRY(hipEventCreate(&b->ev1));
  }
  ts::TsParams TP = b->TP;
  bk::BkParams BP = b->BP;
  HIP_TRY(ctx_next(b->ctx, tsp ? &TP.next : &BP.next));
  HIP_TRY(hipEventRecord(b->ev0, b->ctx->stream));
  uint8_t* mem = (uint8_t*)pool;
  hipStream_t st = b->ctx->stream;
  if (tsp && tr)
    HIP_TRY(launch_ts_replay_episodes(TP, *tr, n, mem, b->bk_bytes, lanes, rec_dev, sum_dev, st));
  else if (tsp)
    HIP_TRY(launch_ts_run_episodes(TP, b->cfg.seed, first, n, mem, b->bk_bytes, lanes, rec_dev,
                                   sum_dev, st));
  else if (tr)
    HIP_TRY(launch_bk_replay_episodes(BP, *tr, n, mem, b->bk_bytes, lanes, rec_dev, sum_dev, st));
  else
    HIP_TRY(launch_bk_run_episodes(BP, b->cfg.seed, first, n, mem, b->bk_bytes, lanes, rec_dev,
                                   sum_dev, st));
  HIP_TRY(hipEventRecord(b->ev1, b->ctx->stream));
  return CPR_OK;
}

// tr == NULL: episodes [first, first + n) of the keyed stream; else trace episodes [0, n)
// FC16 abstract-model episodes: grid-stride over n, a few resident workgroups per CU
static int run_async_fc16(cpr_batch* b, int64_t n, uint64_t first, const TraceSource* tr,
                          cpr_summary* sum_dev, cpr_episode_record* rec_dev) {
  if (tr) return fail(CPR_E_UNSUPPORTED, "FC16 episodes have no trace format");
  int64_t lanes = std::min<int64_t>((int64_t)b->ctx->cus * 8 * 256, ((n + 255) / 256) * 256);
  lanes = std::max<int64_t>(256, lanes);
  if (!b->ev0) {
    HIP_TRY(hipEventCreate(&b->ev0));
    HIP_TRY(hipEventCreate(&b->ev1));
  }
  HIP_TRY(hipEventRecord(b->ev0, b->ctx->stream));
  HIP_TRY(launch_fc16_episodes(b->FP, b->cfg.seed, first, n, lanes, rec_dev, sum_dev,
                               b->ctx->stream));
  HIP_TRY(hipEventRecord(b->ev1, b->ctx->stream));
  return CPR_OK;
}

static int run_async(cpr_batch* b, int64_t n, uint64_t first, const TraceSource* tr,
                     cpr_summary* sum_dev, cpr_episode_record* rec_dev) {
  if (b->cfg.protocol == CPR_PROTO_FC16) return run_async_fc16(b, n, first, tr, sum_dev, rec_dev);
  if (b->cfg.protocol == CPR_PROTO_ETHEREUM || b->nak_ev)
    return run_async_eth(b, n, first, tr, sum_dev, rec_dev);
  if (b->is_ev) return run_async_bk(b, n, first, tr, sum_dev, rec_dev);
  const int64_t lanes = episode_lanes(b, n, rec_dev != nullptr);
  b->last_lanes = lanes;
  b->last_resident =
      (int64_t)b->ctx->cus * run_episodes_blocks_per_cu(b->P, b->cfg.mode, rec_dev != nullptr) * 256;
  // spill [lane][cap] f64 mining times | tie-replay scratch [lane] | the deferred-race
  // kernel's second-pass list (1 + n words)
  const size_t o_replay = align256((size_t)lanes * b->P.cap * sizeof(double));
  const size_t o_list = align256(o_replay + (size_t)lanes * REPLAY_BYTES);
  const size_t list_bytes = tr ? 0 : (size_t)run_episodes_list_bytes(b->P, b->cfg.mode,
                                                                      rec_dev != nullptr, n);
  // the second pass of a deferred-race launch runs on the side stream (cpr_ctx.side) with
  // its list in one of the context's two list buffers; CPR_SIDE_PASS=0 keeps it on the
  // stream with the list in the pool (A/B)
  const char* sp = getenv("CPR_SIDE_PASS");
  const bool side = list_bytes > 0 && !(sp && sp[0] == '0');
  cpr_ctx* c = b->ctx;
  void* pool = nullptr;
  HIP_TRY(ctx_pool(c, side ? o_list : o_list + list_bytes, &pool));
  double* spill = (double*)pool;
  uint8_t* replay = (uint8_t*)pool + o_replay;
  int64_t* list = list_bytes ? (int64_t*)((uint8_t*)pool + o_list) : nullptr;
  const int li = c->list_i;
  if (side) {
    if (c->list_pending[li]) {
      // the pass that reads this buffer (two launches ago) must be done before the main
      // kernel rewrites it; before a reallocation, on the host
      if (c->lists[li].bytes < list_bytes) HIP_TRY(hipEventSynchronize(c->list_ev[li]));
      HIP_TRY(hipStreamWaitEvent(c->stream, c->list_ev[li], 0));
      c->list_pending[li] = false;
    }
    HIP_TRY(c->lists[li].ensure(list_bytes));
    list = (int64_t*)c->lists[li].p;
  }
  if (!b->ev0) {
    HIP_TRY(hipEventCreate(&b->ev0));
    HIP_TRY(hipEventCreate(&b->ev1));
  }
  int64_t* redo = nullptr;
  uint32_t* redo_n = nullptr;
  uint32_t launch_id = 0;
  uint8_t* ovf = nullptr;
  if (b->has_rerun) {
    // hybrid re-runs (nak_hybrid.h) where a quiescent point has the reference's queue state:
    // gym episodes on the selfish-mining network whose attacker messages arrive (gamma > 0),
    // ended by max_steps alone, the whole episode in the engine's block ring, a seeded
    // stream and a deterministic policy; CPR_RERUN_HYBRID=0 re-runs whole episodes (A/B)
    const char* hv = getenv("CPR_RERUN_HYBRID");
    const bool hyb = !(hv && hv[0] == '0') && !tr && b->cfg.mode == CPR_MODE_GYM &&
                     b->cfg.network == CPR_NET_SELFISH_MINING && b->P.arrive == 1 &&
                     !b->P.abstract_g && b->cfg.policy != CPR_POLICY_RANDOM &&
                     !(b->P.max_progress < __builtin_inf()) &&
                     !(b->P.max_time < __builtin_inf()) &&
                     b->NEP.max_steps < (1 << 20) &&
                     b->NEP.max_steps + 2 <= (int64_t)b->NEP.cap_b;
    NakParams NP = b->P;
    NP.cap = (int32_t)((b->NEP.max_steps + 2 + 63) / 64 * 64);
    const int rc = register_rerun(b, b->NEP, b->nak_bytes, first, tr, rec_dev, sum_dev, n,
                                  &redo, &redo_n, &launch_id, &ovf, hyb ? &NP : nullptr);
    if (rc) return rc;
  }
  HIP_TRY(hipEventRecord(b->ev0, b->ctx->stream));
  if (tr)
    HIP_TRY(launch_replay_episodes(b->P, *tr, n, b->cfg.mode, b->cfg.activations,
                                   spill, replay, lanes, rec_dev, sum_dev, redo, redo_n,
                                   launch_id, b->ctx->rq_cap, ovf, b->ctx->stream));
  else {
    // the fused kernel's work queue (kernels.hip nak_next_episode); CPR_NAK_WQ=0 keeps the
    // static grid stride (A/B)
    NakParams P = b->P;
    const char* wq = getenv("CPR_NAK_WQ");
    if (!(wq && wq[0] == '0')) HIP_TRY(ctx_next(b->ctx, &P.next));
    bool ran = false;
    const SidePass sd{c->side, c->main_ev, c->list_ev[li], &ran};
    HIP_TRY(launch_run_episodes(P, b->cfg.seed, first, n, b->cfg.mode, b->cfg.activations,
                                spill, replay, list, lanes, rec_dev, sum_dev, redo, redo_n,
                                launch_id, b->ctx->rq_cap, ovf, b->ctx->stream,
                                side ? &sd : nullptr));
    if (ran) {
      c->list_pending[li] = true;
      c->list_i ^= 1;
      // the launch's time spans both kernels: ev0 on the stream, ev1 behind the second pass
      HIP_TRY(hipEventRecord(b->ev1, c->side));
      return CPR_OK;
    }
  }
  HIP_TRY(hipEventRecord(b->ev1, b->ctx->stream));
  return CPR_OK;
}

int cpr_run_episodes_async(cpr_batch* b, int64_t n, uint64_t first, cpr_summary* sum_dev,
                           cpr_episode_record* rec_dev) {
  if (!b || !sum_dev) return fail(CPR_E_INVALID_ARG, "NULL argument");
  if (n <= 0) return CPR_OK;
  HIP_TRY(hipSetDevice(b->ctx->device));
  b->async_launch = true;
  return run_async(b, n, first, nullptr, sum_dev, rec_dev);
}

static int run_sync(cpr_batch* b, int64_t n, uint64_t first, const TraceSource* tr,
                    cpr_summary* summary, cpr_episode_record* records, int records_on_device) {
  hipStream_t st = b->ctx->stream;
  HIP_TRY(b->summary.ensure(sizeof(cpr_summary)));
  HIP_TRY(hipMemsetAsync(b->summary.p, 0, sizeof(cpr_summary), st));
  cpr_episode_record* rec_dev = nullptr;
  if (records) {
    if (records_on_device)
      rec_dev = records;
    else {
      HIP_TRY(b->records.ensure((size_t)n * sizeof(cpr_episode_record)));
      rec_dev = (cpr_episode_record*)b->records.p;
    }
  }
  int rc = run_async(b, n, first, tr, (cpr_summary*)b->summary.p, rec_dev);
  if (rc) return rc;
  rc = flush_reruns(b->ctx);
  if (rc) return rc;
  cpr_summary s;
  HIP_TRY(hipMemcpyAsync(&s, b->summary.p, sizeof(s), hipMemcpyDeviceToHost, st));
  if (records && !records_on_device)
    HIP_TRY(hipMemcpyAsync(records, rec_dev, (size_t)n * sizeof(cpr_episode_record),
                           hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  float ms = 0.f;
  HIP_TRY(hipEventElapsedTime(&ms, b->ev0, b->ev1));
  b->last_ms = ms;
  b->last_acts = s.activations;
  summary->episodes += s.episodes;
  summary->steps += s.steps;
  summary->activations += s.activations;
  summary->reward_attacker_fx += s.reward_attacker_fx;
  summary->reward_defender_fx += s.reward_defender_fx;
  summary->progress_fx += s.progress_fx;
  summary->rel_revenue_fx += s.rel_revenue_fx;
  summary->rel_revenue_sq_fx += s.rel_revenue_sq_fx;
  summary->orphans += s.orphans;
  summary->status_tie += s.status_tie;
  summary->status_overlap += s.status_overlap;
  summary->status_other += s.status_other;
  summary->invalid += s.invalid;
  for (int i = 0; i < CPR_HIST_BINS; i++) summary->hist[i] += s.hist[i];
  return CPR_OK;
}

int cpr_run_episodes(cpr_batch* b, int64_t n, uint64_t first, cpr_summary* summary,
                     cpr_episode_record* records, int records_on_device) {
  if (!b || !summary) return fail(CPR_E_INVALID_ARG, "NULL argument");
  if (n <= 0) return CPR_OK;
  HIP_TRY(hipSetDevice(b->ctx->device));
  return run_sync(b, n, first, nullptr, summary, records, records_on_device);
}

// host-side checks of a trace before any of it reaches a lane: CSR offsets, miners within
// the network, delays non-negative (not NaN), keys strictly ascending per episode
static int check_trace(const cpr_batch* b, const cpr_trace* t) {
  const int64_t E = t->n_episodes;
  // two agents: 2 nodes; honest clique: exactly `defenders` nodes; selfish mining: the
  // attacker plus `defenders`
  const int32_t nodes = b->cfg.network == CPR_NET_TWO_AGENTS      ? 2
                        : b->cfg.network == CPR_NET_HONEST_CLIQUE ? b->cfg.defenders
                                                                  : b->cfg.defenders + 1;
  const int64_t* offs[3] = {t->act_offset, t->pow_offset, t->link_offset};
  const char* names[3] = {"act_offset", "pow_offset", "link_offset"};
  for (int a = 0; a < 3; a++) {
    const int64_t* o = offs[a];
    const std::string nm = std::string("cpr_trace.") + names[a];
    if (!o) return fail(CPR_E_INVALID_ARG, nm + " is NULL");
    if (o[0] != 0) return fail(CPR_E_INVALID_ARG, nm + "[0] != 0");
    for (int64_t e = 0; e < E; e++)
      if (o[e + 1] < o[e] || o[e + 1] - o[e] > INT32_MAX)
        return fail(CPR_E_INVALID_ARG, nm + " not monotone");
  }
  const int64_t na = t->act_offset[E], np = t->pow_offset[E], nl = t->link_offset[E];
  if ((na && (!t->act_miner || !t->act_delay)) || (np && !t->pow_hash) ||
      (nl && (!t->link_key || !t->link_delay)))
    return fail(CPR_E_INVALID_ARG, "cpr_trace: NULL array with nonzero length");
  for (int64_t i = 0; i < na; i++) {
    if (t->act_miner[i] < 0 || t->act_miner[i] >= nodes)
      return fail(CPR_E_INVALID_ARG, "cpr_trace.act_miner: node index out of range");
    if (!(t->act_delay[i] >= 0.0))
      return fail(CPR_E_INVALID_ARG, "cpr_trace.act_delay: negative or NaN delay");
  }
  for (int64_t i = 0; i < nl; i++)
    if (!(t->link_delay[i] >= 0.0))
      return fail(CPR_E_INVALID_ARG, "cpr_trace.link_delay: negative or NaN delay");
  for (int64_t e = 0; e < E; e++)
    for (int64_t i = t->link_offset[e] + 1; i < t->link_offset[e + 1]; i++)
      if (t->link_key[i] <= t->link_key[i - 1])
        return fail(CPR_E_INVALID_ARG, "cpr_trace.link_key: not strictly ascending");
  return CPR_OK;
}

// copy a checked trace into the batch's trace buffers (on the context's stream)
static int upload_trace(cpr_batch* b, const cpr_trace* t, TraceSource* out) {
  hipStream_t st = b->ctx->stream;
  const int64_t E = t->n_episodes;
  const int64_t na = t->act_offset[E], np = t->pow_offset[E], nl = t->link_offset[E];
  const size_t ob = (size_t)(E + 1) * sizeof(int64_t);
  // one device buffer holds the three offset arrays; empty arrays get 8 bytes
  HIP_TRY(b->tr_off.ensure(3 * ob));
  HIP_TRY(b->tr_miner.ensure(std::max<size_t>(8, (size_t)na * sizeof(int32_t))));
  HIP_TRY(b->tr_delay.ensure(std::max<size_t>(8, (size_t)na * sizeof(double))));
  HIP_TRY(b->tr_pow.ensure(std::max<size_t>(8, (size_t)np * sizeof(int32_t))));
  HIP_TRY(b->tr_key.ensure(std::max<size_t>(8, (size_t)nl * sizeof(uint64_t))));
  HIP_TRY(b->tr_ldelay.ensure(std::max<size_t>(8, (size_t)nl * sizeof(double))));
  char* off = (char*)b->tr_off.p;
  HIP_TRY(hipMemcpyAsync(off, t->act_offset, ob, hipMemcpyHostToDevice, st));
  HIP_TRY(hipMemcpyAsync(off + ob, t->pow_offset, ob, hipMemcpyHostToDevice, st));
  HIP_TRY(hipMemcpyAsync(off + 2 * ob, t->link_offset, ob, hipMemcpyHostToDevice, st));
  if (na) {
    HIP_TRY(hipMemcpyAsync(b->tr_miner.p, t->act_miner, na * sizeof(int32_t),
                           hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(b->tr_delay.p, t->act_delay, na * sizeof(double),
                           hipMemcpyHostToDevice, st));
  }
  if (np)
    HIP_TRY(hipMemcpyAsync(b->tr_pow.p, t->pow_hash, np * sizeof(int32_t), hipMemcpyHostToDevice,
                           st));
  if (nl) {
    HIP_TRY(hipMemcpyAsync(b->tr_key.p, t->link_key, nl * sizeof(uint64_t),
                           hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(b->tr_ldelay.p, t->link_delay, nl * sizeof(double),
                           hipMemcpyHostToDevice, st));
  }
  TraceSource src;
  src.act_off = (const int64_t*)off;
  src.pow_off = (const int64_t*)(off + ob);
  src.link_off = (const int64_t*)(off + 2 * ob);
  src.act_miner = (const int32_t*)b->tr_miner.p;
  src.act_delay = (const double*)b->tr_delay.p;
  src.pow_hash = (const int32_t*)b->tr_pow.p;
  src.link_key = (const uint64_t*)b->tr_key.p;
  src.link_delay = (const double*)b->tr_ldelay.p;
  *out = src;
  return CPR_OK;
}

int cpr_replay(cpr_batch* b, const cpr_trace* t, cpr_summary* summary,
               cpr_episode_record* records, int records_on_device) {
  if (!b || !t || !summary) return fail(CPR_E_INVALID_ARG, "NULL argument");
  if (b->cfg.network == CPR_NET_ABSTRACT_GAMMA)
    return fail(CPR_E_UNSUPPORTED, "the abstract-gamma mode has no trace replay");
  if (t->n_episodes <= 0) return CPR_OK;
  int rc = check_trace(b, t);
  if (rc) return rc;
  HIP_TRY(hipSetDevice(b->ctx->device));
  TraceSource src;
  rc = upload_trace(b, t, &src);
  if (rc) return rc;
  return run_sync(b, t->n_episodes, 0, &src, summary, records, records_on_device);
}

static int32_t network_nodes(const cpr_config& c) {
  return c.network == CPR_NET_TWO_AGENTS      ? 2
         : c.network == CPR_NET_HONEST_CLIQUE ? c.defenders
                                               : c.defenders + 1;  // attacker + defenders
}

// Per-node outputs (csv_runner.ml:74-79): the episodes run once more on the exact event
// engine with a second per-lane region holding activations per node and per-block reward
// arrays; Nakamoto configurations of the closed-form lane use the Nakamoto-mode engine of
// the exact re-runs (same episodes, bit for bit)
int cpr_node_outputs(cpr_batch* b, int64_t n, uint64_t first, const cpr_trace* trace,
                     int32_t n_nodes, cpr_episode_record* records, int64_t* node_activations,
                     double* node_rewards) {
  if (!b || !node_activations || !node_rewards) return fail(CPR_E_INVALID_ARG, "NULL argument");
  if (b->cfg.protocol == CPR_PROTO_FC16)
    return fail(CPR_E_UNSUPPORTED, "FC16 episodes have no network nodes");
  if (b->cfg.network == CPR_NET_ABSTRACT_GAMMA)
    return fail(CPR_E_UNSUPPORTED, "the abstract-gamma mode has no exact event engine");
  if (n_nodes != network_nodes(b->cfg))
    return fail(CPR_E_INVALID_ARG, "n_nodes must equal the network's node count");
  const bool nak_fused = b->cfg.protocol == CPR_PROTO_NAKAMOTO && !b->nak_ev;
  if (nak_fused && !b->has_rerun)
    return fail(CPR_E_UNSUPPORTED, "configuration beyond the exact event engine's capacity");
  int rc;
  TraceSource src;
  if (trace) {
    rc = check_trace(b, trace);
    if (rc) return rc;
    n = trace->n_episodes;
    first = 0;
  }
  if (n <= 0) return CPR_OK;
  HIP_TRY(hipSetDevice(b->ctx->device));
  if (trace) {
    rc = upload_trace(b, trace, &src);
    if (rc) return rc;
  }
  hipStream_t st = b->ctx->stream;
  const bool eth = b->cfg.protocol == CPR_PROTO_ETHEREUM || b->cfg.protocol == CPR_PROTO_NAKAMOTO;
  const bool tsp = b->cfg.protocol == CPR_PROTO_TAILSTORM;
  eth::EthParams EP = nak_fused ? b->NEP : b->EP;
  ts::TsParams TP = b->TP;
  bk::BkParams BP = b->BP;
  const int64_t lane_bytes = eth ? eth::eth_lane_bytes(EP.cap_b, EP.cap_e, EP.n) : b->bk_bytes;
  const int64_t node_bytes = eth ? eth::eth_node_bytes(EP.cap_b, EP.n)
                             : tsp ? ts::ts_align((int64_t)b->TP.n * 8)
                                   : bk::bk_node_bytes(b->BP);
  const int64_t per_cu = eth ? eth_blocks_per_cu() : (tsp ? ts_blocks_per_cu() : bk_blocks_per_cu());
  const int64_t full = (int64_t)b->ctx->cus * per_cu * 256;
  const int64_t budget = kLaneBudget / (lane_bytes + node_bytes);
  int64_t lanes = std::min(full, std::max<int64_t>(256, budget));
  lanes = std::min(lanes, ((n + 255) / 256) * 256);
  lanes = std::max<int64_t>(256, (lanes / 256) * 256);
  void* pool = nullptr;
  const size_t o_node = align256((size_t)lanes * (size_t)lane_bytes);
  HIP_TRY(ctx_pool(b->ctx, o_node + (size_t)lanes * (size_t)node_bytes, &pool));
  DevBuf out, sum;
  const size_t rows = (size_t)n * (size_t)n_nodes;
  const size_t o_rew = align256(rows * 8), o_hm = o_rew + align256(rows * 8),
               o_rec = o_hm + align256((size_t)n * 4);
  HIP_TRY(out.ensure(o_rec + (size_t)n * sizeof(cpr_episode_record)));
  HIP_TRY(sum.ensure(sizeof(cpr_summary)));
  HIP_TRY(hipMemsetAsync(sum.p, 0, sizeof(cpr_summary), st));
  NodeOut no;
  no.mem = (uint8_t*)pool + o_node;
  no.lane_bytes = node_bytes;
  no.acts = (int64_t*)out.p;
  no.rews = (double*)((char*)out.p + o_rew);
  no.head_miner = (int32_t*)((char*)out.p + o_hm);
  cpr_episode_record* rec = (cpr_episode_record*)((char*)out.p + o_rec);
  cpr_summary* sd = (cpr_summary*)sum.p;
  uint8_t* mem = (uint8_t*)pool;
  HIP_TRY(ctx_next(b->ctx, eth ? &EP.next : tsp ? &TP.next : &BP.next));
  if (eth && trace)
    HIP_TRY(launch_eth_replay_episodes(EP, src, n, mem, lane_bytes, lanes, rec, sd, st, no));
  else if (eth)
    HIP_TRY(launch_eth_run_episodes(EP, b->cfg.seed, first, n, mem, lane_bytes, lanes, rec, sd,
                                    st, no));
  else if (tsp && trace)
    HIP_TRY(launch_ts_replay_episodes(TP, src, n, mem, lane_bytes, lanes, rec, sd, st, no));
  else if (tsp)
    HIP_TRY(launch_ts_run_episodes(TP, b->cfg.seed, first, n, mem, lane_bytes, lanes, rec, sd,
                                   st, no));
  else if (trace)
    HIP_TRY(launch_bk_replay_episodes(BP, src, n, mem, lane_bytes, lanes, rec, sd, st, no));
  else
    HIP_TRY(launch_bk_run_episodes(BP, b->cfg.seed, first, n, mem, lane_bytes, lanes, rec, sd,
                                   st, no));
  std::vector<int32_t> hm((size_t)n);
  HIP_TRY(hipMemcpyAsync(node_activations, no.acts, rows * 8, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipMemcpyAsync(node_rewards, no.rews, rows * 8, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipMemcpyAsync(hm.data(), no.head_miner, (size_t)n * 4, hipMemcpyDeviceToHost, st));
  if (records)
    HIP_TRY(hipMemcpyAsync(records, rec, (size_t)n * sizeof(cpr_episode_record),
                           hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  if (records)
    for (int64_t e = 0; e < n; e++) records[e].head_miner = hm[(size_t)e];
  return CPR_OK;
}

// ---------------------------------------------------------------- lockstep API

static int obs_len_of(const cpr_config& c) {
  switch (c.protocol) {
    case CPR_PROTO_BK: return 8;
    case CPR_PROTO_ETHEREUM: return 10;
    case CPR_PROTO_TAILSTORM: return 10;
    default: return 4;
  }
}

static int ensure_common_lockstep(cpr_batch* b, int obs_len) {
  const int64_t n = b->cfg.n_lanes;
  HIP_TRY(b->l_obs.ensure((size_t)n * obs_len * sizeof(double)));
  HIP_TRY(b->l_act.ensure((size_t)n * sizeof(int32_t)));
  HIP_TRY(b->l_rew.ensure((size_t)n * sizeof(double)));
  HIP_TRY(b->l_done.ensure((size_t)n));
  HIP_TRY(b->l_mask.ensure((size_t)n));
  HIP_TRY(b->l_eps.ensure((size_t)n * sizeof(uint64_t)));
  HIP_TRY(b->l_info.ensure((size_t)n * (7 * 8 + 3 * 4)));
  return CPR_OK;
}

// per-lane region bytes of the event-engine lockstep lanes (B_k, Tailstorm, Ethereum)
static int64_t ev_lane_bytes(const cpr_batch* b) { return b->is_eth ? b->eth_bytes : b->bk_bytes; }

static int ensure_lockstep_bk(cpr_batch* b) {
  const int64_t n = b->cfg.n_lanes;
  if (n <= 0) return fail(CPR_E_STATE, "batch has no lockstep lanes (cfg.n_lanes = 0)");
  if (b->cfg.mode != CPR_MODE_GYM) return fail(CPR_E_STATE, "lockstep lanes need CPR_MODE_GYM");
  if (!b->bk_slots.p) {
    HIP_TRY(b->bk_lmem.ensure((size_t)n * (size_t)ev_lane_bytes(b)));
    const size_t sb = b->is_eth ? eth_slot_bytes()
                      : b->cfg.protocol == CPR_PROTO_TAILSTORM ? ts_slot_bytes() : bk_slot_bytes();
    HIP_TRY(b->bk_slots.ensure((size_t)n * sb));
    HIP_TRY(hipMemsetAsync(b->bk_slots.p, 0, (size_t)n * sb, b->ctx->stream));
  }
  return ensure_common_lockstep(b, obs_len_of(b->cfg));
}

static int ensure_lockstep(cpr_batch* b) {
  if (b->is_ev || b->is_eth) return ensure_lockstep_bk(b);
  const int64_t n = b->cfg.n_lanes;
  if (n <= 0) return fail(CPR_E_STATE, "batch has no lockstep lanes (cfg.n_lanes = 0)");
  if (b->cfg.mode != CPR_MODE_GYM) return fail(CPR_E_STATE, "lockstep lanes need CPR_MODE_GYM");
  if (!b->lanes.p) {
    HIP_TRY(b->lanes.ensure((size_t)n * lock_lane_bytes()));
    HIP_TRY(hipMemsetAsync(b->lanes.p, 0, (size_t)n * lock_lane_bytes(), b->ctx->stream));
  }
  if (b->has_rerun && !b->l_alog.p) {
    // lanes leaving the closed form continue on the exact engine: an action log of the
    // episode so far and event-engine lanes handed out on first need and returned at the
    // lane's next reset. Every lane gets a slot and a log of its whole episode when they
    // fit the budgets (kExactSlotBudget of slots: 65,536 lanes of 2,016-step episodes
    // take ~27 GB of the 288 GB; kActionLogBudget of logs), so the lockstep API stays
    // exact for every lane like engine.ml's step (engine.ml:176-249); beyond the budgets
    // (lanes x episode length), a lane that finds no slot keeps the closed form's flags.
    // The slot pool is also capped at a quarter of the device's free memory, and an
    // allocation that fails is retried with half the slots (down to 256) instead of failing
    // the reset: at the gym's delays almost no lane ever leaves the closed form
    constexpr int64_t kExactSlotBudget = 48ll << 30, kActionLogBudget = 4ll << 30;
    const int64_t ms = b->P.max_steps > 0 && b->P.max_steps < (1ll << 30) ? b->P.max_steps
                                                                          : (1 << 14);
    int64_t cap = std::min<int64_t>(ms, kActionLogBudget / n);
    cap = std::max<int64_t>(1, cap);
    b->alog_cap = cap;
    const int64_t eb = std::max<int64_t>(1, b->nak_bytes);
    int64_t slots = std::min<int64_t>(n, std::max<int64_t>(256, kExactSlotBudget / eb));
    size_t free_b = 0, total_b = 0;
    if (hipMemGetInfo(&free_b, &total_b) == hipSuccess)
      slots = std::min<int64_t>(slots, std::max<int64_t>(256, (int64_t)(free_b / 4) / eb));
    slots = std::min<int64_t>(slots, n);
    HIP_TRY(b->l_alog.ensure((size_t)n * (size_t)cap));
    for (;;) {
      const hipError_t e = b->l_emem.ensure((size_t)slots * (size_t)eb);
      if (e == hipSuccess) break;
      (void)hipGetLastError();
      if (slots <= 256) HIP_TRY(e);
      slots = std::max<int64_t>(256, slots / 2);
    }
    b->n_exact_slots = (int32_t)slots;
    HIP_TRY(b->l_eslots.ensure((size_t)b->n_exact_slots * sizeof(eth::EthLane)));
    std::vector<int32_t> stack((size_t)b->n_exact_slots + 1);
    for (int32_t i = 0; i < b->n_exact_slots; i++) stack[i] = i;
    stack[b->n_exact_slots] = b->n_exact_slots;  // stack height: every slot free
    HIP_TRY(b->l_efree.ensure(stack.size() * 4));
    HIP_TRY(hipMemcpy(b->l_efree.p, stack.data(), stack.size() * 4, hipMemcpyHostToDevice));
  }
  HIP_TRY(b->lring.ensure((size_t)n * RING * sizeof(double)));
  HIP_TRY(b->lspill.ensure((size_t)n * b->P.cap * sizeof(double)));
  HIP_TRY(b->lreplay.ensure((size_t)n * REPLAY_BYTES));
  HIP_TRY(b->l_obs.ensure((size_t)n * 4 * sizeof(double)));
  HIP_TRY(b->l_act.ensure((size_t)n * sizeof(int32_t)));
  HIP_TRY(b->l_rew.ensure((size_t)n * sizeof(double)));
  HIP_TRY(b->l_done.ensure((size_t)n));
  HIP_TRY(b->l_mask.ensure((size_t)n));
  HIP_TRY(b->l_eps.ensure((size_t)n * sizeof(uint64_t)));
  HIP_TRY(b->l_info.ensure((size_t)n * (7 * 8 + 3 * 4)));
  return CPR_OK;
}

static LockBuffers lock_buffers(cpr_batch* b) {
  LockBuffers B;
  B.lanes = b->lanes.p;
  B.ring = (double*)b->lring.p;
  B.spill = (double*)b->lspill.p;
  B.replay = (uint8_t*)b->lreplay.p;
  B.alog = (uint8_t*)b->l_alog.p;
  B.alog_cap = b->alog_cap;
  B.emem = (uint8_t*)b->l_emem.p;
  B.elane_bytes = b->nak_bytes;
  B.eslots = b->l_eslots.p;
  B.efree = (int32_t*)b->l_efree.p;
  B.n_slots = b->n_exact_slots;
  return B;
}

int cpr_reset(cpr_batch* b, const uint8_t* mask, const uint64_t* eps, double* obs) {
  if (!b || !obs) return fail(CPR_E_INVALID_ARG, "NULL argument");
  if (b->cfg.protocol == CPR_PROTO_FC16)
    return fail(CPR_E_UNSUPPORTED, "FC16 runs fused episodes (cpr_run_episodes) only");
  HIP_TRY(hipSetDevice(b->ctx->device));
  int rc = ensure_lockstep(b);
  if (rc) return rc;
  const int64_t n = b->cfg.n_lanes;
  hipStream_t st = b->ctx->stream;
  if (!b->reset_done && mask) {
    for (int64_t i = 0; i < n; i++)
      if (!mask[i]) return fail(CPR_E_STATE, "first reset must include every lane");
  }
  const uint8_t* dmask = nullptr;
  const uint64_t* deps = nullptr;
  if (mask) {
    HIP_TRY(hipMemcpyAsync(b->l_mask.p, mask, (size_t)n, hipMemcpyHostToDevice, st));
    dmask = (const uint8_t*)b->l_mask.p;
  }
  if (eps) {
    HIP_TRY(hipMemcpyAsync(b->l_eps.p, eps, (size_t)n * 8, hipMemcpyHostToDevice, st));
    deps = (const uint64_t*)b->l_eps.p;
  }
  const double* tabs = (const double*)b->tabs_dev.p;
  const int ol = obs_len_of(b->cfg);
  if (b->is_eth)
    HIP_TRY(launch_eth_reset(b->EP, b->cfg.seed, (uint8_t*)b->bk_lmem.p, b->eth_bytes,
                             b->bk_slots.p, n, dmask, deps, b->cfg.unit_observation, tabs,
                             b->tab_n, (double*)b->l_obs.p, st));
  else if (b->cfg.protocol == CPR_PROTO_BK)
    HIP_TRY(launch_bk_reset(b->BP, b->cfg.seed, (uint8_t*)b->bk_lmem.p, b->bk_bytes,
                            b->bk_slots.p, n, dmask, deps, b->cfg.unit_observation, tabs,
                            b->tab_n, (double*)b->l_obs.p, st));
  else if (b->cfg.protocol == CPR_PROTO_TAILSTORM)
    HIP_TRY(launch_ts_reset(b->TP, b->cfg.seed, (uint8_t*)b->bk_lmem.p, b->bk_bytes,
                            b->bk_slots.p, n, dmask, deps, b->cfg.unit_observation, tabs,
                            b->tab_n, (double*)b->l_obs.p, st));
  else
    HIP_TRY(launch_reset(b->P, b->NEP, b->cfg.seed, lock_buffers(b), n, dmask, deps,
                         b->cfg.unit_observation, tabs, tabs + b->tab_n, b->tab_n,
                         (double*)b->l_obs.p, st));
  HIP_TRY(hipMemcpyAsync(obs, b->l_obs.p, (size_t)n * ol * sizeof(double), hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  b->reset_done = true;
  return CPR_OK;
}

int cpr_step(cpr_batch* b, const int32_t* actions, double* obs, double* reward, uint8_t* done,
             cpr_step_info* info) {
  if (!b || !actions || !obs || !reward || !done) return fail(CPR_E_INVALID_ARG, "NULL argument");
  if (!b->reset_done) return fail(CPR_E_STATE, "step before reset");
  const int64_t n = b->cfg.n_lanes;
  const int n_act = b->is_eth ? 24 : b->is_ev ? 8 : 4;
  const int ol = obs_len_of(b->cfg);
  for (int64_t i = 0; i < n; i++)
    if (actions[i] < 0 || actions[i] >= n_act)
      return fail(CPR_E_INVALID_ARG, "Invalid_argument \"index out of bounds\" (action)");
  HIP_TRY(hipSetDevice(b->ctx->device));
  hipStream_t st = b->ctx->stream;
  HIP_TRY(hipMemcpyAsync(b->l_act.p, actions, (size_t)n * 4, hipMemcpyHostToDevice, st));
  char* ib = (char*)b->l_info.p;
  StepBuffers sb;
  sb.obs = (double*)b->l_obs.p;
  sb.reward = (double*)b->l_rew.p;
  sb.done = (uint8_t*)b->l_done.p;
  sb.era = (double*)(ib);
  sb.erd = (double*)(ib + n * 8);
  sb.eprog = (double*)(ib + 2 * n * 8);
  sb.ect = (double*)(ib + 3 * n * 8);
  sb.est = (double*)(ib + 4 * n * 8);
  sb.esteps = (int64_t*)(ib + 5 * n * 8);
  sb.eacts = (int64_t*)(ib + 6 * n * 8);
  sb.hh = (int32_t*)(ib + 7 * n * 8);
  sb.hm = (int32_t*)(ib + 7 * n * 8 + n * 4);
  sb.status = (uint32_t*)(ib + 7 * n * 8 + 2 * n * 4);
  const double* tabs = (const double*)b->tabs_dev.p;
  if (b->is_eth)
    HIP_TRY(launch_eth_step(b->EP, b->cfg.seed, (uint8_t*)b->bk_lmem.p, b->eth_bytes,
                            b->bk_slots.p, n, (const int32_t*)b->l_act.p,
                            b->cfg.unit_observation, tabs, b->tab_n, sb, st));
  else if (b->cfg.protocol == CPR_PROTO_BK)
    HIP_TRY(launch_bk_step(b->BP, b->cfg.seed, (uint8_t*)b->bk_lmem.p, b->bk_bytes,
                           b->bk_slots.p, n, (const int32_t*)b->l_act.p,
                           b->cfg.unit_observation, tabs, b->tab_n, sb, st));
  else if (b->cfg.protocol == CPR_PROTO_TAILSTORM)
    HIP_TRY(launch_ts_step(b->TP, b->cfg.seed, (uint8_t*)b->bk_lmem.p, b->bk_bytes,
                           b->bk_slots.p, n, (const int32_t*)b->l_act.p,
                           b->cfg.unit_observation, tabs, b->tab_n, sb, st));
  else
  {
    const LockBuffers LB = lock_buffers(b);
    HIP_TRY(launch_step(b->P, b->cfg.seed, LB, n, (const int32_t*)b->l_act.p,
                        b->cfg.unit_observation, tabs, tabs + b->tab_n, b->tab_n, sb, st));
    HIP_TRY(launch_lock_exact(b->NEP, b->cfg.seed, LB, n, (const int32_t*)b->l_act.p,
                              b->cfg.unit_observation, tabs, tabs + b->tab_n, b->tab_n, sb, st));
  }
  HIP_TRY(hipMemcpyAsync(obs, sb.obs, (size_t)n * ol * 8, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipMemcpyAsync(reward, sb.reward, (size_t)n * 8, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipMemcpyAsync(done, sb.done, (size_t)n, hipMemcpyDeviceToHost, st));
  if (info) {
    struct {
      void* dst;
      void* src;
      size_t sz;
    } cp[] = {{info->episode_reward_attacker, sb.era, 8},  {info->episode_reward_defender, sb.erd, 8},
              {info->episode_progress, sb.eprog, 8},       {info->episode_chain_time, sb.ect, 8},
              {info->episode_sim_time, sb.est, 8},         {info->episode_n_steps, sb.esteps, 8},
              {info->episode_n_activations, sb.eacts, 8},  {info->head_height, sb.hh, 4},
              {info->head_miner, sb.hm, 4},                {info->status, sb.status, 4}};
    for (auto& x : cp)
      if (x.dst) HIP_TRY(hipMemcpyAsync(x.dst, x.src, (size_t)n * x.sz, hipMemcpyDeviceToHost, st));
  }
  HIP_TRY(hipStreamSynchronize(st));
  return CPR_OK;
}

int cpr_observe_fields(cpr_batch* b, int32_t* fields) {
  if (!b || !fields) return fail(CPR_E_INVALID_ARG, "NULL argument");
  if (!b->reset_done) return fail(CPR_E_STATE, "observe before reset");
  const int64_t n = b->cfg.n_lanes;
  HIP_TRY(hipSetDevice(b->ctx->device));
  hipStream_t st = b->ctx->stream;
  const size_t per = (size_t)obs_len_of(b->cfg) * 4;
  DevBuf tmp;
  HIP_TRY(tmp.ensure((size_t)n * per));
  if (b->is_eth)
    HIP_TRY(launch_eth_observe_fields(b->EP, (uint8_t*)b->bk_lmem.p, b->eth_bytes, b->bk_slots.p,
                                      n, (int32_t*)tmp.p, st));
  else if (b->cfg.protocol == CPR_PROTO_BK)
    HIP_TRY(launch_bk_observe_fields(b->BP, (uint8_t*)b->bk_lmem.p, b->bk_bytes, b->bk_slots.p,
                                     n, (int32_t*)tmp.p, st));
  else if (b->cfg.protocol == CPR_PROTO_TAILSTORM)
    HIP_TRY(launch_ts_observe_fields(b->TP, (uint8_t*)b->bk_lmem.p, b->bk_bytes, b->bk_slots.p,
                                     n, (int32_t*)tmp.p, st));
  else
    HIP_TRY(launch_observe_fields(b->NEP, lock_buffers(b), n, (int32_t*)tmp.p, st));
  HIP_TRY(hipMemcpyAsync(fields, tmp.p, (size_t)n * per, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  tmp.release();
  return CPR_OK;
}

int cpr_policy_actions(cpr_batch* b, int32_t policy, const double* obs, int64_t n,
                       int32_t* actions) {
  if (!b || !obs || !actions) return fail(CPR_E_INVALID_ARG, "NULL argument");
  if (b->cfg.protocol == CPR_PROTO_TAILSTORM) {
    if (policy < 0 || policy > CPR_TS_POLICY_TABLE)
      return fail(CPR_E_INVALID_ARG, "unknown policy");
    if (policy == CPR_TS_POLICY_TABLE && b->table_host.empty())
      return fail(CPR_E_INVALID_ARG, "batch has no policy table");
    if (n <= 0) return CPR_OK;
    HIP_TRY(hipSetDevice(b->ctx->device));
    hipStream_t st = b->ctx->stream;
    DevBuf& o = b->pol_obs;
    DevBuf& a = b->pol_act;
    HIP_TRY(o.ensure((size_t)n * 80));
    HIP_TRY(a.ensure((size_t)n * 4));
    HIP_TRY(hipMemcpyAsync(o.p, obs, (size_t)n * 80, hipMemcpyHostToDevice, st));
    HIP_TRY(launch_ts_policy(policy, b->cfg.k, b->cfg.unit_observation, (const double*)o.p, n,
                             (const uint8_t*)b->table_dev.p, b->cfg.policy_table_dim,
                             (int32_t*)a.p, st));
    HIP_TRY(hipMemcpyAsync(actions, a.p, (size_t)n * 4, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    return CPR_OK;
  }
  if (b->cfg.protocol == CPR_PROTO_BK) {
    if (policy < 0 || policy > CPR_BK_POLICY_TABLE) return fail(CPR_E_INVALID_ARG, "unknown policy");
    if (policy == CPR_BK_POLICY_TABLE && b->table_host.empty())
      return fail(CPR_E_INVALID_ARG, "batch has no policy table");
    if (n <= 0) return CPR_OK;
    HIP_TRY(hipSetDevice(b->ctx->device));
    hipStream_t st = b->ctx->stream;
    DevBuf& o = b->pol_obs;
    DevBuf& a = b->pol_act;
    HIP_TRY(o.ensure((size_t)n * 64));
    HIP_TRY(a.ensure((size_t)n * 4));
    HIP_TRY(hipMemcpyAsync(o.p, obs, (size_t)n * 64, hipMemcpyHostToDevice, st));
    bk::BkParams P = b->BP;
    P.policy = policy;
    HIP_TRY(launch_bk_policy(P, b->cfg.unit_observation, (const double*)o.p, n, (int32_t*)a.p, st));
    HIP_TRY(hipMemcpyAsync(actions, a.p, (size_t)n * 4, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    return CPR_OK;
  }
  if (b->is_eth) {
    if (policy < 0 || policy > CPR_ETH_POLICY_TABLE)
      return fail(CPR_E_INVALID_ARG, "unknown policy");
    if (policy == CPR_ETH_POLICY_TABLE && b->table_host.empty())
      return fail(CPR_E_INVALID_ARG, "batch has no policy table");
    if (n <= 0) return CPR_OK;
    HIP_TRY(hipSetDevice(b->ctx->device));
    hipStream_t st = b->ctx->stream;
    DevBuf& o = b->pol_obs;
    DevBuf& a = b->pol_act;
    HIP_TRY(o.ensure((size_t)n * 80));
    HIP_TRY(a.ensure((size_t)n * 4));
    HIP_TRY(hipMemcpyAsync(o.p, obs, (size_t)n * 80, hipMemcpyHostToDevice, st));
    HIP_TRY(launch_eth_policy(policy, b->cfg.unit_observation, (const double*)o.p, n,
                              (const uint8_t*)b->table_dev.p, b->cfg.policy_table_dim,
                              (int32_t*)a.p, st));
    HIP_TRY(hipMemcpyAsync(actions, a.p, (size_t)n * 4, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    return CPR_OK;
  }
  if (b->cfg.protocol != CPR_PROTO_NAKAMOTO)
    return fail(CPR_E_UNSUPPORTED, "policy evaluation on encoded observations");
  if (policy < 0 || policy > CPR_POLICY_TABLE) return fail(CPR_E_INVALID_ARG, "unknown policy");
  if (policy == CPR_POLICY_TABLE && b->table_host.empty())
    return fail(CPR_E_INVALID_ARG, "batch has no policy table");
  if (n <= 0) return CPR_OK;
  HIP_TRY(hipSetDevice(b->ctx->device));
  hipStream_t st = b->ctx->stream;
  DevBuf& o = b->pol_obs;
  DevBuf& a = b->pol_act;
  HIP_TRY(o.ensure((size_t)n * 32));
  HIP_TRY(a.ensure((size_t)n * 4));
  HIP_TRY(hipMemcpyAsync(o.p, obs, (size_t)n * 32, hipMemcpyHostToDevice, st));
  HIP_TRY(launch_policy(policy, b->cfg.unit_observation, (const double*)o.p, n,
                        (const uint8_t*)b->table_dev.p, b->cfg.policy_table_dim, (int32_t*)a.p,
                        st));
  HIP_TRY(hipMemcpyAsync(actions, a.p, (size_t)n * 4, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  return CPR_OK;
}

// ssz_tools.ml:64-73 ranges; nakamoto_ssz.ml:43-61
int cpr_observation_spec(cpr_batch* b, int32_t* obs_len, int32_t* n_actions, double* low,
                         double* high) {
  if (!b) return fail(CPR_E_INVALID_ARG, "NULL argument");
  const double inf = __builtin_inf();
  if (b->cfg.protocol == CPR_PROTO_FC16) {
    // fc16.rs:61-73: (a, h, fork index) each mapped x -> x / (1 + x); at most 4 actions
    if (obs_len) *obs_len = 3;
    if (n_actions) *n_actions = 4;
    for (int i = 0; i < 3; i++) {
      if (low) low[i] = 0.0;
      if (high) high[i] = 1.0;
    }
    return CPR_OK;
  }
  if (b->cfg.protocol == CPR_PROTO_TAILSTORM) {
    // tailstorm_ssz.ml:41-79: 10 fields (diff signed, event discrete), Action8
    if (obs_len) *obs_len = 10;
    if (n_actions) *n_actions = 8;
    for (int i = 0; i < 10; i++) {
      double lo = 0.0, hi = 1.0;
      if (!b->cfg.unit_observation) {
        lo = i == 2 ? -inf : 0.0;
        hi = i == 9 ? 2.0 : inf;
      }
      if (low) low[i] = lo;
      if (high) high[i] = hi;
    }
    return CPR_OK;
  }
  if (b->cfg.protocol == CPR_PROTO_BK) {
    // bk_ssz.ml:37-74 normalizers; ssz_tools.ml:64-74 ranges (raw Bool range is (0, 0))
    if (obs_len) *obs_len = 8;
    if (n_actions) *n_actions = 8;
    for (int i = 0; i < 8; i++) {
      double lo = 0.0, hi = 1.0;
      if (!b->cfg.unit_observation) {
        lo = i == 2 ? -inf : 0.0;
        hi = i == 6 ? 0.0 : (i == 7 ? 2.0 : inf);
      }
      if (low) low[i] = lo;
      if (high) high[i] = hi;
    }
    return CPR_OK;
  }
  if (b->cfg.protocol == CPR_PROTO_ETHEREUM) {
    // ethereum_ssz.ml:47-80: 10 fields (diff_* signed, event discrete), 24 actions
    if (obs_len) *obs_len = 10;
    if (n_actions) *n_actions = 24;
    for (int i = 0; i < 10; i++) {
      const bool sgn = i == 4 || i == 5;
      double lo = 0.0, hi = 1.0;
      if (!b->cfg.unit_observation && i != 9) {
        lo = sgn ? -inf : 0.0;
        hi = inf;
      }
      if (low) low[i] = lo;
      if (high) high[i] = hi;
    }
    return CPR_OK;
  }
  if (obs_len) *obs_len = 4;
  if (n_actions) *n_actions = 4;
  if (b->cfg.unit_observation) {
    for (int i = 0; i < 4; i++) {
      if (low) low[i] = 0.0;
      if (high) high[i] = 1.0;
    }
  } else {
    const double lo[4] = {0.0, 0.0, -inf, 0.0}, hi[4] = {inf, inf, inf, 1.0};
    for (int i = 0; i < 4; i++) {
      if (low) low[i] = lo[i];
      if (high) high[i] = hi[i];
    }
  }
  return CPR_OK;
}

// Collection.add prepends (collection.ml:13): registry order is the reverse of the adds
// in nakamoto_ssz.ml:342-350
static const char* kNames[4] = {"sapirshtein-2016-sm1", "eyal-sirer-2014", "simple", "honest"};
static const int32_t kIds[4] = {CPR_POLICY_SAPIRSHTEIN_2016_SM1, CPR_POLICY_EYAL_SIRER_2014,
                                CPR_POLICY_SIMPLE, CPR_POLICY_HONEST};

// ethereum_ssz.ml:523-538, same reversal
static const char* kEthNames[5] = {"fn19pkel", "fn19", "selfish_discard", "selfish_release",
                                   "honest"};
static const int32_t kEthIds[5] = {CPR_ETH_POLICY_FN19PKEL, CPR_ETH_POLICY_FN19,
                                   CPR_ETH_POLICY_SELFISH_DISCARD,
                                   CPR_ETH_POLICY_SELFISH_RELEASE, CPR_ETH_POLICY_HONEST};

// bk_ssz.ml:404-415, same reversal
static const char* kBkNames[4] = {"avoid-loss", "minor-delay", "get-ahead", "honest"};
static const int32_t kBkIds[4] = {CPR_BK_POLICY_AVOID_LOSS, CPR_BK_POLICY_MINOR_DELAY,
                                  CPR_BK_POLICY_GET_AHEAD, CPR_BK_POLICY_HONEST};

// tailstorm_ssz.ml:449-472, same reversal
static const char* kTsNames[7] = {"long-delay", "avoid-loss-b", "avoid-loss-a", "avoid-loss",
                                  "minor-delay", "get-ahead", "honest"};
static const int32_t kTsIds[7] = {CPR_TS_POLICY_LONG_DELAY, CPR_TS_POLICY_AVOID_LOSS_B,
                                  CPR_TS_POLICY_AVOID_LOSS_A, CPR_TS_POLICY_AVOID_LOSS,
                                  CPR_TS_POLICY_MINOR_DELAY, CPR_TS_POLICY_GET_AHEAD,
                                  CPR_TS_POLICY_HONEST};

int cpr_policy_count(int32_t protocol) {
  switch (protocol) {
    case CPR_PROTO_NAKAMOTO: return 4;
    case CPR_PROTO_ETHEREUM: return 5;
    case CPR_PROTO_BK: return 4;
    case CPR_PROTO_TAILSTORM: return 7;
    default: return 0;
  }
}

const char* cpr_policy_name(int32_t protocol, int32_t index, int32_t* policy_id) {
  if (index < 0 || index >= cpr_policy_count(protocol)) {
    g_err = "no such policy";
    return nullptr;
  }
  if (protocol == CPR_PROTO_ETHEREUM) {
    if (policy_id) *policy_id = kEthIds[index];
    return kEthNames[index];
  }
  if (protocol == CPR_PROTO_BK) {
    if (policy_id) *policy_id = kBkIds[index];
    return kBkNames[index];
  }
  if (protocol == CPR_PROTO_TAILSTORM) {
    if (policy_id) *policy_id = kTsIds[index];
    return kTsNames[index];
  }
  if (policy_id) *policy_id = kIds[index];
  return kNames[index];
}

int cpr_rollout(cpr_batch* b, int64_t n_steps, double* obs, double* reward, uint8_t* done,
                int outputs_on_device, cpr_summary* summary) {
  if (!b || !summary) return fail(CPR_E_INVALID_ARG, "NULL argument");
  if (!b->is_ev && !b->is_eth)
    return fail(CPR_E_UNSUPPORTED, "cpr_rollout is implemented for Ethereum, B_k and Tailstorm");
  if (n_steps <= 0) return CPR_OK;
  HIP_TRY(hipSetDevice(b->ctx->device));
  int rc = ensure_lockstep(b);
  if (rc) return rc;
  hipStream_t st = b->ctx->stream;
  HIP_TRY(b->summary.ensure(sizeof(cpr_summary)));
  HIP_TRY(hipMemsetAsync(b->summary.p, 0, sizeof(cpr_summary), st));
  if (!b->ev0) {
    HIP_TRY(hipEventCreate(&b->ev0));
    HIP_TRY(hipEventCreate(&b->ev1));
  }
  const int64_t cells = n_steps * b->cfg.n_lanes;
  const int ol = obs_len_of(b->cfg);
  double* obs_dev = obs;
  double* reward_dev = reward;
  uint8_t* done_dev = done;
  DevBuf so, sr, sd;
  if (!outputs_on_device) {
    if (obs) {
      HIP_TRY(so.ensure((size_t)cells * ol * 8));
      obs_dev = (double*)so.p;
    }
    if (reward) {
      HIP_TRY(sr.ensure((size_t)cells * 8));
      reward_dev = (double*)sr.p;
    }
    if (done) {
      HIP_TRY(sd.ensure((size_t)cells));
      done_dev = (uint8_t*)sd.p;
    }
  }
  const double* tabs = (const double*)b->tabs_dev.p;
  HIP_TRY(hipEventRecord(b->ev0, st));
  if (b->is_eth)
    HIP_TRY(launch_eth_rollout(b->EP, b->cfg.seed, (uint8_t*)b->bk_lmem.p, b->eth_bytes,
                               b->bk_slots.p, b->cfg.n_lanes, n_steps, b->cfg.unit_observation,
                               tabs, b->tab_n, obs_dev, reward_dev, done_dev,
                               (cpr_summary*)b->summary.p, st));
  else if (b->cfg.protocol == CPR_PROTO_TAILSTORM)
    HIP_TRY(launch_ts_rollout(b->TP, b->cfg.seed, (uint8_t*)b->bk_lmem.p, b->bk_bytes,
                              b->bk_slots.p, b->cfg.n_lanes, n_steps, b->cfg.unit_observation,
                              tabs, b->tab_n, obs_dev, reward_dev, done_dev,
                              (cpr_summary*)b->summary.p, st));
  else
    HIP_TRY(launch_bk_rollout(b->BP, b->cfg.seed, (uint8_t*)b->bk_lmem.p, b->bk_bytes,
                              b->bk_slots.p, b->cfg.n_lanes, n_steps, b->cfg.unit_observation,
                              tabs, b->tab_n, obs_dev, reward_dev, done_dev,
                              (cpr_summary*)b->summary.p, st));
  HIP_TRY(hipEventRecord(b->ev1, st));
  cpr_summary s;
  HIP_TRY(hipMemcpyAsync(&s, b->summary.p, sizeof(s), hipMemcpyDeviceToHost, st));
  if (!outputs_on_device) {
    if (obs) HIP_TRY(hipMemcpyAsync(obs, obs_dev, (size_t)cells * ol * 8, hipMemcpyDeviceToHost, st));
    if (reward) HIP_TRY(hipMemcpyAsync(reward, reward_dev, (size_t)cells * 8, hipMemcpyDeviceToHost, st));
    if (done) HIP_TRY(hipMemcpyAsync(done, done_dev, (size_t)cells, hipMemcpyDeviceToHost, st));
  }
  HIP_TRY(hipStreamSynchronize(st));
  so.release();
  sr.release();
  sd.release();
  float ms = 0.f;
  HIP_TRY(hipEventElapsedTime(&ms, b->ev0, b->ev1));
  b->last_ms = ms;
  b->last_acts = s.activations;
  b->reset_done = true;
  // rollout lanes are the batch's n_lanes (one thread each, 256-thread workgroups); the
  // resident figure is the fused-episode kernel's occupancy of the same lane
  b->last_lanes = b->cfg.n_lanes;
  b->last_resident = (int64_t)b->ctx->cus * 256 *
                     (b->is_eth ? eth_blocks_per_cu()
                                : (b->cfg.protocol == CPR_PROTO_TAILSTORM ? ts_blocks_per_cu()
                                                                          : bk_blocks_per_cu()));
  summary->episodes += s.episodes;
  summary->steps += s.steps;
  summary->activations += s.activations;
  summary->reward_attacker_fx += s.reward_attacker_fx;
  summary->reward_defender_fx += s.reward_defender_fx;
  summary->progress_fx += s.progress_fx;
  summary->rel_revenue_fx += s.rel_revenue_fx;
  summary->rel_revenue_sq_fx += s.rel_revenue_sq_fx;
  summary->orphans += s.orphans;
  summary->status_tie += s.status_tie;
  summary->status_overlap += s.status_overlap;
  summary->status_other += s.status_other;
  summary->invalid += s.invalid;
  for (int i = 0; i < CPR_HIST_BINS; i++) summary->hist[i] += s.hist[i];
  return CPR_OK;
}

int cpr_stream_fill(cpr_ctx* ctx, uint64_t seed, uint64_t ep, uint32_t idx0, uint32_t tag,
                    int64_t n, uint32_t* out, double* exp_out) {
  if (!ctx || !out) return fail(CPR_E_INVALID_ARG, "NULL argument");
  if (n <= 0) return CPR_OK;
  HIP_TRY(hipSetDevice(ctx->device));
  DevBuf o, e;
  HIP_TRY(o.ensure((size_t)n * 16));
  if (exp_out) HIP_TRY(e.ensure((size_t)n * 8));
  HIP_TRY(launch_stream_fill(seed, ep, idx0, tag, n, (uint32_t*)o.p, (double*)e.p, ctx->stream));
  HIP_TRY(hipMemcpyAsync(out, o.p, (size_t)n * 16, hipMemcpyDeviceToHost, ctx->stream));
  if (exp_out)
    HIP_TRY(hipMemcpyAsync(exp_out, e.p, (size_t)n * 8, hipMemcpyDeviceToHost, ctx->stream));
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  o.release();
  e.release();
  return CPR_OK;
}

}  // extern "C"

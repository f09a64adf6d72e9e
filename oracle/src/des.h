// TEST INFRASTRUCTURE ONLY — CPU oracle (faithful restatement of the reference DES).
//
// This is the checker for libcpr_hip, never the thing measured or shipped. It restates
// the OCaml discrete-event simulator of pkel/cpr function by function:
//   OrderedQueue (skew heap)        simulator/lib/orderedQueue.ml:17-47
//   Dag (vertices, children order)  simulator/lib/dag.ml:1-45
//   Distributions (alias, exp, uni) simulator/lib/distributions.ml:12-98
//   Network topologies              simulator/lib/network.ml:36-105
//   Simulator (events, visibility)  simulator/lib/simulator.ml:122-543
//   Dagtools.common_ancestor        simulator/lib/dagtools.ml:73-121
//   Nakamoto referee / honest node  simulator/protocols/nakamoto.ml:19-96
//   SSZ'16 attack space + policies  simulator/protocols/nakamoto_ssz.ml:23-350
//   Gym engine (reset/step/info)    simulator/gym/engine.ml:97-273
// Randomness: either the OCaml 4.12 `Random` replica (sequential, reproduces the
// reference's recorded outputs) or the keyed Philox stream shared with the GPU.
#pragma once
#include <cstdint>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "keyed_stream.h"
#include "ocaml_random.h"

namespace oracle {

enum VisKind : uint8_t { INVISIBLE = 0, RECEIVED, RELEASED, WITHHELD };
struct Vis {
  VisKind kind = INVISIBLE;
  double time = 0.0;
};

// block payload: Nakamoto {height; miner} (nakamoto.ml:8-12); Ethereum adds work
// (ethereum.ml:69-73, always 0 for Nakamoto); B_k: kind 1 = Vote {height; id = miner},
// kind 0 = Block {height} with miner -1 (bk.ml:26-35)
struct NakData {
  int height = 0;
  int miner = -1;  // -1 = None
  int work = 0;
  int kind = 0;
  bool operator==(const NakData& o) const {
    return height == o.height && miner == o.miner && work == o.work && kind == o.kind;
  }
};

struct Block {
  int serial = 0;
  std::vector<Block*> parents;
  std::vector<Block*> children_app;  // append order; Dag's list is newest first
  int depth = 0;
  NakData value;
  bool has_pow = false;
  int32_t pow_hash = 0;
  int signature = -1;
  std::vector<Vis> vis;
  std::vector<double> received_at;
  std::vector<double> rewards;
  // keyed-stream coordinates of the message (set when the block is shared)
  int share_k = -1;
  int share_off = 0;
};

// Ethereum referee pieces (ethereum.cpp): validity (ethereum.ml:102-151, Byzantium
// max_uncles = 2) and the Constant / Discount reward functions (ethereum.ml:173-197)
bool eth_validity(const Block* b);
void eth_reward(const Block* x, int scheme, std::vector<double>& r);
// B_k referee pieces (bk.cpp): validity (bk.ml:110-132), Constant / Block rewards
// (bk.ml:151-176)
bool bk_validity(const Block* b, int k);
void bk_reward(const Block* x, int scheme, int k, std::vector<double>& r);
// Tailstorm referee pieces (tailstorm.cpp): validity (tailstorm.ml:156-180), rewards
// (tailstorm.ml:204-233)
bool ts_validity(const Block* b, int k);
void ts_reward(const Block* x, int scheme, int k, std::vector<double>& r);

struct Draft {
  std::vector<Block*> parents;
  NakData data;
  bool sign = false;
};

enum EvType { EV_CLOCK, EV_DAG, EV_NET_TX, EV_NET_RX, EV_ONNODE, EV_MAKEVIS, EV_MADEVIS };
enum Kind { K_APPEND = 0, K_POW = 1, K_NETWORK = 2 };

struct Event {
  EvType type;
  int node;
  Kind kind;
  Block* blk;
  int draft;
};

// persistent skew heap of orderedQueue.ml, implemented in place (old versions are never
// reused by the simulator, so in-place mutation is observationally identical)
struct SkewHeap {
  struct N {
    double t;
    int ev;
    int l, r;
  };
  std::vector<N> pool;
  std::vector<int> freelist;
  int root = -1;
  int len = 0;
  void clear() { pool.clear(); freelist.clear(); root = -1; len = 0; }
  int alloc(double t, int ev);
  int ins(int node, double t, int ev);
  int remove_top(int node);
  void queue(double t, int ev) { root = ins(root, t, ev); len++; }
  bool dequeue(double* t, int* ev);
};

int float_compare(double a, double b);  // OCaml Float.compare

enum DelayKind { D_CONST, D_UNIFORM, D_EXP };
struct Link {
  int dest;
  DelayKind kind;
  double a, b;  // const: a; uniform: [a, b); exp: ev = a
};
struct NetNode {
  double compute;
  std::vector<Link> links;
};
struct Network {
  std::vector<NetNode> nodes;
  bool flooding = false;
  double activation_delay = 1.0;
  // network.ml:50-59
  static Network two_agents(double activation_delay, double alpha);
  // network.ml:61-105 (raises on defenders < 2 or gamma > (d-1)/d)
  static Network selfish_mining(double alpha, double activation_delay, double gamma,
                                double propagation_delay, int defenders);
};

struct SimRng {
  virtual ~SimRng() {}
  virtual int miner(int k) = 0;
  virtual double act_delay(int j) = 0;
  virtual int32_t pow_bits(int serial) = 0;
  virtual double link_delay(const Link& l, const Block* msg) = 0;
  // abstract-gamma coin of defender j for the release shared at activation count kw
  // (CPR_NET_ABSTRACT_GAMMA; keyed stream only)
  virtual double coin(int kw, int j) {
    (void)kw;
    (void)j;
    throw std::runtime_error("abstract-gamma coins need the keyed stream");
  }
  // the i-th random attacker action among n (the `random` policy of the reference's policy
  // tests, cpr_protocols.ml:658-782: Random.int A.Action.n at every decision)
  virtual int rand_action(int i, int n) {
    (void)i;
    (void)n;
    throw std::runtime_error("random attacker actions need the keyed or OCaml stream");
  }
};

// OCaml Random: alias sampling exactly as distributions.ml:45-98
struct OcamlSimRng : SimRng {
  OcamlRandom* r;
  std::vector<double> p;
  std::vector<int> alias;
  double ev;
  OcamlSimRng(OcamlRandom* r, const Network& net);
  int miner(int k) override;
  double act_delay(int j) override;
  int32_t pow_bits(int serial) override;
  double link_delay(const Link& l, const Block* msg) override;
  int rand_action(int, int n) override { return r->int_(n); }  // Random.int, in stream order
};

// keyed Philox stream (keyed_stream.h); weights must be [alpha, equal rest]
struct KeyedSimRng : SimRng {
  KeyedStream ks;
  uint64_t t_att;
  int d;
  double ev;
  bool serial_links = false;  // key link delays by (message serial, dest): TAG_MSG
  std::vector<uint32_t> thr;  // general_weights: keyed miner thresholds (honest cliques)
  KeyedSimRng(uint64_t seed, uint64_t episode, const Network& net, bool general_weights = false);
  int miner(int k) override;
  double act_delay(int j) override;
  int32_t pow_bits(int serial) override;
  double link_delay(const Link& l, const Block* msg) override;
  double coin(int kw, int j) override { return ks.link_u((uint32_t)kw, 0u, (uint32_t)j); }
  int rand_action(int i, int n) override { return ks.rand_action((uint32_t)i, n); }
};

// keyed miner draw by general weights iff the compute is not [alpha] + equal defenders
// summing to 1 (honest cliques of models.ml:3-28: compute 1..n, also for n = 2); the
// two-agents and symmetric-clique networks keep the two-threshold draw
inline bool needs_general_weights(const Network& net) {
  double total = 0.0;
  for (const NetNode& x : net.nodes) total += x.compute;
  if (total > 1.0 + 1e-9 || total < 1.0 - 1e-9) return true;
  for (size_t i = 2; i < net.nodes.size(); ++i)
    if (net.nodes[i].compute != net.nodes[1].compute) return true;
  return false;
}

// ---- activation/delay traces (cpr_trace, include/cpr_hip.h)
// One episode's draws addressed by keyed-stream coordinates: activation j's miner and
// clock delay, vertex serial s's pow bits, message delays by link key (kw, off, dest) or,
// for B_k / Tailstorm, by message key (serial, dest). Constant-delay links draw nothing.
struct TraceBuf {
  std::vector<int32_t> miner;
  std::vector<double> delay;
  std::vector<int32_t> pow;
  std::map<uint64_t, double> link;
  uint32_t miss = 0;  // replay: a draw the trace does not hold
};
enum { TRACE_OFF = 0, TRACE_RECORD = 1, TRACE_REPLAY = 2 };
// per-thread hook consulted wherever an episode builds its SimRng: RECORD wraps the rng
// (or, with `ocaml` set, an OcamlSimRng on that shared state) and logs every draw into
// `buf`; REPLAY draws from `buf` instead
struct TraceHook {
  int mode = TRACE_OFF;
  TraceBuf* buf = nullptr;
  OcamlRandom* ocaml = nullptr;
};
extern thread_local TraceHook g_trace;
uint64_t trace_link_key(uint32_t kw, uint32_t off, uint32_t dest);
uint64_t trace_msg_key(uint32_t serial, uint32_t dest);
std::unique_ptr<SimRng> trace_wrap(std::unique_ptr<SimRng> inner, const Network& net,
                                   bool serial_links);

struct Sim;

struct Action {
  std::vector<Block*> share;
  std::vector<Draft> append;
};

struct NodeImpl {
  Sim* sim = nullptr;
  int id = 0;
  virtual ~NodeImpl() {}
  virtual Draft puzzle_payload() = 0;
  virtual Action handler(Kind k, Block* b) = 0;
  virtual Block* preferred() = 0;
};

// diagnostics (not part of the reference; used to audit the GPU lane machine)
enum : uint32_t {
  DIAG_TIE = 1u,      // a defender saw two equal-height candidates at the same instant
  DIAG_OVERLAP = 2u,  // an activation fired while finite-time messages were in flight
};

struct Sim {
  double now = 0.0;
  SkewHeap queue;
  int c_activations = 0;
  std::vector<Event> events;
  std::vector<Draft> drafts;
  std::vector<std::unique_ptr<Block>> dag;
  std::vector<Block*> roots;  // Dag.roots order (newest first)
  std::vector<std::unique_ptr<NodeImpl>> nodes;
  std::vector<int> activations;
  Network net;
  SimRng* rng;
  int n_nodes = 0;
  uint32_t diag = 0;
  int pending_finite_rx = 0;
  // protocol of the referee: 0 = Nakamoto, 1 = Ethereum (Byzantium parameters), 2 = B_k,
  // 3 = Tailstorm (bk_k = k, bk_scheme = the Tailstorm incentive scheme)
  int proto = 0;
  int eth_scheme = 0;  // Ethereum incentive scheme: 0 = Constant, 1 = Discount
  int bk_k = 0;        // B_k votes per block
  // guard (not in the reference): appends allowed between two activations; 0 = no limit.
  // A B_k attacker policy that keeps adopting re-proposes on the same block at the same
  // instant forever, which Simulator.loop (no step bound) would never leave.
  int zt_limit = 0;
  int zt_appends = 0;
  int bk_scheme = 0;   // B_k incentive scheme: 0 = Constant, 2 = Block

  Sim(const Network& net, SimRng* rng);
  void init(std::vector<std::unique_ptr<NodeImpl>> nodes_);
  void schedule(double delay, const Event& ev);
  void schedule_now(const Event& ev) { schedule(0.0, ev); }
  void schedule_pow();
  bool visible(int node, const Block* b) const { return b->vis[node].kind != INVISIBLE; }
  Block* raw_append(bool pow, int node, const Draft& d);
  Block* append(bool pow, int node, const Draft& d);
  void handle_action(int node, const Action& act);
  void handle_event(const Event& ev);
  bool dequeue(Event* ev);
  void loop(int activations);
  Block* head();
  // referee: Nakamoto (nakamoto.ml:19-57) or Ethereum (ethereum.ml:89-199)
  bool validity(const Block* b) const;
  void reward(Block* x) const;  // set_rewards (simulator.ml:377-388)
  double progress(const Block* b) const {
    if (proto == 2)  // bk.ml:42-46
      return (double)(b->value.height * bk_k + (b->value.kind == 1 ? 1 : 0));
    if (proto == 3)  // tailstorm.ml:72: height * k + depth
      return (double)(b->value.height * bk_k + (b->value.kind == 1 ? b->value.work : 0));
    return proto == 1 ? (double)b->value.work : (double)b->value.height;
  }
  // nakamoto.ml:43-48 and ethereum.ml:159-162 (both: first maximum height)
  static Block* winner(const std::vector<Block*>& l);
  static double timestamp(const Block* b);
};

// Dagtools.common_ancestor over node `view`'s parents (dagtools.ml:102-121)
Block* common_ancestor(const Sim& sim, int view, Block* a, Block* b);

struct NakHonest : NodeImpl {
  Block* state = nullptr;
  // CPR_NET_ABSTRACT_GAMMA (not the reference; a flagged mode of the build): a release by
  // node 0 that ties a defender block mined at this instant wins iff coin < abstract_gamma
  double abstract_gamma = -1.0;
  Draft puzzle_payload() override;
  Action handler(Kind k, Block* b) override;
  Block* preferred() override { return state; }
};

enum Policy { POL_HONEST = 0, POL_SIMPLE = 1, POL_ES2014 = 2, POL_SM1 = 3, POL_TABLE = 4,
              POL_RANDOM = 5 };
// nakamoto_ssz.ml:116-154 — Variants.to_rank
enum NakAction { ADOPT = 0, OVERRIDE = 1, MATCH = 2, WAIT = 3 };

struct NakObs {
  int public_blocks, private_blocks, diff_blocks, event;  // event: 0 PoW, 1 Network
};

struct TablePolicy {
  int dim = 0;                  // observation clamp
  std::vector<uint8_t> actions; // [(pub * dim + priv) * 2 + event]
};

int nak_policy(int policy, const NakObs& o, const TablePolicy* table);
void nak_obs_to_floats(const NakObs& o, bool unit, double out[4]);
NakObs nak_obs_of_floats(const double in[4], bool unit);

// nakamoto_ssz.ml Agent (:256-360)
struct NakSszAgent {
  Sim* sim = nullptr;
  int my_id = 0;
  Block* pub = nullptr;
  Block* priv = nullptr;
  std::vector<Block*> pending;
  // observable state
  Block* o_pub = nullptr;
  Block* o_priv = nullptr;
  Block* o_common = nullptr;
  int o_event = 0;
  void init(Block* root) { pub = priv = root; pending.clear(); }
  Draft puzzle_payload() const;
  void prepare(Kind k, Block* x);
  NakObs observe() const;
  Action apply(int action);
};

// attacker as a simulator node (nakamoto_ssz.ml:262-272), used by Simulator.loop tasks
struct NakSszAttackerNode : NodeImpl {
  NakSszAgent agent;
  int policy;
  int nrand = 0;  // POL_RANDOM decisions so far
  const TablePolicy* table = nullptr;
  Draft puzzle_payload() override { return agent.puzzle_payload(); }
  Action handler(Kind k, Block* b) override;
  Block* preferred() override { return agent.priv; }
};

// engine.ml:82-95
struct DummyNode : NodeImpl {
  Block* state = nullptr;
  Draft puzzle_payload() override;
  Action handler(Kind, Block*) override;
  Block* preferred() override { return state; }
};

struct GymParams {
  double alpha = 0.25, gamma = 0.5;
  int defenders = 2;
  double activation_delay = 1.0;
  long max_steps = 0x3fffffffffffffffL;
  double max_progress = 1.0 / 0.0;
  double max_time = 1.0 / 0.0;
  bool unit_obs = true;
  // defender<->defender delay of Network.T.selfish_mining; the gym passes 1e-9
  // (engine.ml:100-107), other values exercise overlapping delivery windows in tests
  double propagation_delay = 1e-9;
  // flagged abstract-gamma mode (include/cpr_hip.h CPR_NET_ABSTRACT_GAMMA): zero delays,
  // match races decided by per-defender coins < gamma
  bool abstract_gamma = false;
};

struct StepInfo {
  double step_reward_attacker, step_reward_defender, step_progress, step_chain_time,
      step_sim_time;
  double episode_reward_attacker, episode_reward_defender, episode_progress,
      episode_chain_time, episode_sim_time;
  long episode_n_steps, episode_n_activations;
  int head_height, head_miner;  // head_miner -1 = n/a
  int head_work;                // Ethereum head info (ethereum.ml:93-97)
};

// engine.ml of_module for the nakamoto_ssz attack space
struct GymNakamoto {
  GymParams p;
  Network net;
  // rng factory state
  int rng_mode = 0;  // 0 = ocaml (shared), 1 = keyed
  OcamlRandom* ocaml = nullptr;
  uint64_t seed = 0, episode = 0;
  std::unique_ptr<SimRng> rng;
  std::unique_ptr<Sim> sim;
  NakSszAgent agent;
  long episode_steps = 0;
  double last_progress = 0, last_chain_time = 0, last_sim_time = 0, last_reward_attacker = 0,
         last_reward_defender = 0;

  GymNakamoto(const GymParams& p, int rng_mode, OcamlRandom* ocaml, uint64_t seed,
              uint64_t episode);
  void init();
  void reset(double obs[4]);
  void observe(double obs[4]) const;
  NakObs observe_int() const { return agent.observe(); }
  double step(int action, double obs[4], bool* done, StepInfo* info);
  Kind skip_to_interaction(Block** blk);
};

// validation of engine.ml:37-51; returns empty string if ok
std::string gym_params_error(const GymParams& p);

}  // namespace oracle

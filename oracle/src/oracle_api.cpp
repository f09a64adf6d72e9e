// TEST INFRASTRUCTURE ONLY — C entry points of the CPU oracle for tests/ and for
// bench.py's cpu_baseline leg. Never used by the product path.
#include <chrono>
#include <cmath>
#include <cstring>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "../../include/cpr_hip.h"
#include "des.h"
#include "ethereum.h"
#include "bk.h"
#include "tailstorm.h"
#include "ocaml_sort.h"

using namespace oracle;

static thread_local std::string g_err;

static void set_err(const char* what) { g_err = what; }

static EthTable eth_table_of(const cpr_config* c) {
  EthTable t;
  if (c->policy == ETH_POL_TABLE && c->policy_table) {
    t.dim = c->policy_table_dim;
    t.actions.assign(c->policy_table, c->policy_table + (size_t)t.dim * t.dim * 2);
  }
  return t;
}
static TsTable ts_table_of(const cpr_config* c) {
  TsTable t;
  if (c->policy == TS_POL_TABLE && c->policy_table) {
    t.dim = c->policy_table_dim;
    const size_t K1 = (size_t)c->k + 1;
    t.actions.assign(c->policy_table, c->policy_table + (size_t)t.dim * t.dim * K1 * K1 * 3);
  }
  return t;
}


extern "C" {

const char* oracle_last_error() { return g_err.c_str(); }

// ---------------- OCaml Random replica
void* oracle_ocaml_rng_new(long seed) {
  return seed < 0 ? new OcamlRandom() : new OcamlRandom(seed);
}
void oracle_ocaml_rng_free(void* r) { delete (OcamlRandom*)r; }
// an independent copy of the 55-word state (branching a Parany worker's stream)
void* oracle_ocaml_rng_copy(void* r) { return new OcamlRandom(*(OcamlRandom*)r); }
int32_t oracle_ocaml_rng_bits(void* r) { return ((OcamlRandom*)r)->bits(); }
int32_t oracle_ocaml_rng_int(void* r, int32_t n) { return ((OcamlRandom*)r)->int_(n); }
double oracle_ocaml_rng_float(void* r, double b) { return ((OcamlRandom*)r)->float_(b); }

// ---------------- keyed stream
void oracle_keyed_block(uint64_t seed, uint64_t episode, uint32_t idx, uint32_t tag,
                        uint32_t out[4]) {
  KeyedStream(seed, episode).block(idx, tag, out);
}
void oracle_philox_raw(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
  Philox4x32::block(ctr, key, out);
}
double oracle_cpr_log(double x) { return cpr_log(x); }
double oracle_u53(uint32_t a, uint32_t b) { return u53(a, b); }

// ---------------- nakamoto_ssz policies / observation encoding
int oracle_nak_policy(int policy, const int32_t obs[4], const uint8_t* table, int dim) {
  TablePolicy t;
  if (policy == POL_TABLE) {
    t.dim = dim;
    t.actions.assign(table, table + dim * dim * 2);
  }
  NakObs o{obs[0], obs[1], obs[2], obs[3]};
  return nak_policy(policy, o, &t);
}
void oracle_nak_obs_to_floats(const int32_t obs[4], int unit, double out[4]) {
  NakObs o{obs[0], obs[1], obs[2], obs[3]};
  nak_obs_to_floats(o, unit != 0, out);
}
void oracle_nak_obs_of_floats(const double in[4], int unit, int32_t out[4]) {
  NakObs o = nak_obs_of_floats(in, unit != 0);
  out[0] = o.public_blocks;
  out[1] = o.private_blocks;
  out[2] = o.diff_blocks;
  out[3] = o.event;
}

// ---------------- Simulator.loop task on the two-agents network with an SSZ attacker
// (experiments/simulate/models.ml:29-46, withholding.ml:6-27, csv_runner.ml:56-98)
// rng_mode 0: OCaml Random state `rng` (carried over between calls like a Parany worker)
// rng_mode 1: keyed stream (seed, episode)
// Simulator.loop task on experiments/simulate/models.ml:3-28 honest_clique: n honest nodes,
// compute i + 1, links to every other node with uniform [lo, hi) propagation delays,
// simple dissemination. proto 0 Nakamoto, 1 Ethereum (Byzantium, scheme). Keyed mode uses
// the general-weight miner draw (weight_thresholds). Outputs per node (n entries).
int oracle_clique_task(int proto, int rng_mode, void* rng, uint64_t seed, uint64_t episode,
                       int n, double activation_delay, double lo, double hi, int scheme,
                       int activations, int64_t* acts_out, double* rewards_out,
                       double* head_time, double* head_progress, int32_t* head_height,
                       int32_t* head_miner, int32_t* head_work) {
  try {
    Network net;
    net.flooding = false;
    net.activation_delay = activation_delay;
    net.nodes.resize(n);
    for (int i = 0; i < n; ++i) {
      net.nodes[i].compute = (double)(i + 1);
      for (int j = 0; j < n - 1; ++j)
        net.nodes[i].links.push_back(Link{j >= i ? j + 1 : j, D_UNIFORM, lo, hi});
    }
    std::unique_ptr<SimRng> r;
    if (rng_mode == 0)
      r.reset(new OcamlSimRng((OcamlRandom*)rng, net));
    else
      r.reset(new KeyedSimRng(seed, episode, net, true));
    r = trace_wrap(std::move(r), net, false);
    Sim sim(net, r.get());
    std::vector<std::unique_ptr<NodeImpl>> nodes;
    if (proto == 1) {
      sim.proto = 1;
      sim.eth_scheme = scheme;
      for (int i = 0; i < n; ++i) nodes.emplace_back(new EthHonest());
    } else {
      for (int i = 0; i < n; ++i) nodes.emplace_back(new NakHonest());
    }
    sim.init(std::move(nodes));
    Block* root = sim.roots.back();
    for (int i = 0; i < n; ++i) {
      if (proto == 1)
        static_cast<EthHonest*>(sim.nodes[i].get())->state = root;
      else
        static_cast<NakHonest*>(sim.nodes[i].get())->state = root;
    }
    sim.loop(activations);
    Block* h = sim.head();
    for (int i = 0; i < n; i++) {
      acts_out[i] = sim.activations[i];
      rewards_out[i] = h->rewards[i];
    }
    *head_time = Sim::timestamp(h);
    *head_progress = sim.progress(h);
    *head_height = h->value.height;
    *head_miner = h->value.miner;
    *head_work = h->value.work;
    return 0;
  } catch (std::exception& e) {
    set_err(e.what());
    return -1;
  }
}

int oracle_two_agents_task(int rng_mode, void* rng, uint64_t seed, uint64_t episode,
                           double alpha, int policy, int activations, int64_t acts_out[2],
                           double rewards_out[2], double* head_time, double* head_progress,
                           int32_t* head_height, uint32_t* diag) {
  try {
    Network net = Network::two_agents(1.0, alpha);
    std::unique_ptr<SimRng> r;
    if (rng_mode == 0)
      r.reset(new OcamlSimRng((OcamlRandom*)rng, net));
    else
      r.reset(new KeyedSimRng(seed, episode, net));
    r = trace_wrap(std::move(r), net, false);
    Sim sim(net, r.get());
    std::vector<std::unique_ptr<NodeImpl>> nodes;
    auto* att = new NakSszAttackerNode();
    att->policy = policy;
    nodes.emplace_back(att);
    nodes.emplace_back(new NakHonest());
    sim.init(std::move(nodes));
    Block* root = sim.roots.back();
    att->agent.sim = &sim;
    att->agent.my_id = 0;
    att->agent.init(root);
    static_cast<NakHonest*>(sim.nodes[1].get())->state = root;
    sim.loop(activations);
    Block* h = sim.head();
    for (int i = 0; i < 2; i++) {
      acts_out[i] = sim.activations[i];
      rewards_out[i] = h->rewards[i];
    }
    *head_time = Sim::timestamp(h);
    *head_progress = (double)h->value.height;
    *head_height = h->value.height;
    if (diag) *diag = sim.diag;
    return 0;
  } catch (std::exception& e) {
    set_err(e.what());
    return -1;
  }
}

// Simulator.loop task on experiments/simulate/models.ml:54-84 selfish_mining: node 0 the
// nakamoto_ssz attacker (policy), `defenders` honest Nakamoto nodes, Network.T.selfish_mining
// with activation delay 1 and defender message delay msg_delay (the withholding sweep's
// gamma-* rows, withholding.ml:29-52). gamma = 0 keeps the attacker's messages at t = +inf;
// Simulator.loop drains them after the last activation (simulator.ml:519-533). Outputs per
// node (defenders + 1 entries).
int oracle_sm_task(int rng_mode, void* rng, uint64_t seed, uint64_t episode, double alpha,
                   double gamma, int defenders, double msg_delay, int policy, int activations,
                   int64_t* acts_out, double* rewards_out, double* head_time,
                   double* head_progress, int32_t* head_height, int32_t* head_miner,
                   uint32_t* diag) {
  try {
    Network net = Network::selfish_mining(alpha, 1.0, gamma, msg_delay, defenders);
    std::unique_ptr<SimRng> r;
    if (rng_mode == 0)
      r.reset(new OcamlSimRng((OcamlRandom*)rng, net));
    else
      r.reset(new KeyedSimRng(seed, episode, net));
    r = trace_wrap(std::move(r), net, false);
    Sim sim(net, r.get());
    std::vector<std::unique_ptr<NodeImpl>> nodes;
    auto* att = new NakSszAttackerNode();
    att->policy = policy;
    nodes.emplace_back(att);
    for (int i = 0; i < defenders; ++i) nodes.emplace_back(new NakHonest());
    sim.init(std::move(nodes));
    Block* root = sim.roots.back();
    att->agent.sim = &sim;
    att->agent.my_id = 0;
    att->agent.init(root);
    for (int i = 1; i <= defenders; ++i) static_cast<NakHonest*>(sim.nodes[i].get())->state = root;
    sim.loop(activations);
    Block* h = sim.head();
    for (int i = 0; i <= defenders; i++) {
      acts_out[i] = sim.activations[i];
      rewards_out[i] = h->rewards[i];
    }
    *head_time = Sim::timestamp(h);
    *head_progress = (double)h->value.height;
    *head_height = h->value.height;
    *head_miner = h->value.miner;
    if (diag) *diag = sim.diag;
    return 0;
  } catch (std::exception& e) {
    set_err(e.what());
    return -1;
  }
}

// ---------------- gym env handle (engine.ml:97-273 for nakamoto_ssz)
static GymParams params_of(const cpr_config* c) {
  GymParams p;
  p.alpha = c->alpha;
  p.gamma = c->gamma;
  p.defenders = c->defenders;
  p.activation_delay = c->activation_delay;
  p.max_steps = c->max_steps > 0 ? c->max_steps : 0x3fffffffffffffffL;
  p.max_progress = c->max_progress > 0 ? c->max_progress : 1.0 / 0.0;
  p.max_time = c->max_time > 0 ? c->max_time : 1.0 / 0.0;
  p.unit_obs = c->unit_observation != 0;
  if (c->propagation_delay > 0) p.propagation_delay = c->propagation_delay;
  p.abstract_gamma = c->network == CPR_NET_ABSTRACT_GAMMA;
  return p;
}

void* oracle_gym_new(const cpr_config* c, int rng_mode, void* ocaml_rng, uint64_t episode) {
  try {
    return new GymNakamoto(params_of(c), rng_mode, (OcamlRandom*)ocaml_rng, c->seed, episode);
  } catch (std::exception& e) {
    set_err(e.what());
    return nullptr;
  }
}
void oracle_gym_free(void* g) { delete (GymNakamoto*)g; }

int oracle_gym_reset(void* g, double obs[4]) {
  try {
    ((GymNakamoto*)g)->reset(obs);
    return 0;
  } catch (std::exception& e) {
    set_err(e.what());
    return -1;
  }
}

int oracle_gym_obs_fields(void* g, int32_t out[4]) {
  NakObs o = ((GymNakamoto*)g)->observe_int();
  out[0] = o.public_blocks;
  out[1] = o.private_blocks;
  out[2] = o.diff_blocks;
  out[3] = o.event;
  return 0;
}

// info_out: 12 doubles in engine.ml:226-237 order + head_height + head_miner
int oracle_gym_step(void* g, int action, double obs[4], double* reward, int* done,
                    double info_out[14]) {
  try {
    bool d = false;
    StepInfo i;
    *reward = ((GymNakamoto*)g)->step(action, obs, &d, &i);
    *done = d ? 1 : 0;
    if (info_out) {
      double v[14] = {i.step_reward_attacker,    i.step_reward_defender,
                      i.step_progress,           i.step_chain_time,
                      i.step_sim_time,           i.episode_reward_attacker,
                      i.episode_reward_defender, i.episode_progress,
                      i.episode_chain_time,      i.episode_sim_time,
                      (double)i.episode_n_steps, (double)i.episode_n_activations,
                      (double)i.head_height,     (double)i.head_miner};
      memcpy(info_out, v, sizeof(v));
    }
    return 0;
  } catch (std::exception& e) {
    set_err(e.what());
    return -1;
  }
}

uint32_t oracle_gym_diag(void* g) { return ((GymNakamoto*)g)->sim->diag; }

// ---------------- OCaml Array.sort replica (stdlib/array.ml), Int.compare keys
void oracle_ocaml_sort_ints(int32_t* a, int n) {
  std::vector<int32_t> v(a, a + n);
  ocaml_array_sort(v, [](int32_t x, int32_t y) { return x < y ? -1 : (x > y ? 1 : 0); });
  memcpy(a, v.data(), sizeof(int32_t) * n);
}
// sort (key, tag) pairs by key only: exposes the heap sort's order among equal keys
void oracle_ocaml_sort_pairs(int32_t* keys, int32_t* tags, int n) {
  std::vector<std::pair<int32_t, int32_t>> v;
  for (int i = 0; i < n; i++) v.push_back({keys[i], tags[i]});
  ocaml_array_sort(v, [](const std::pair<int32_t, int32_t>& x,
                         const std::pair<int32_t, int32_t>& y) {
    return x.first < y.first ? -1 : (x.first > y.first ? 1 : 0);
  });
  for (int i = 0; i < n; i++) {
    keys[i] = v[i].first;
    tags[i] = v[i].second;
  }
}
int oracle_at_most_first_ints(int32_t* a, int n, int k) {
  std::vector<int32_t> v(a, a + n);
  v = ocaml_at_most_first(v, [](int32_t x, int32_t y) { return x < y ? -1 : (x > y ? 1 : 0); }, k);
  memcpy(a, v.data(), sizeof(int32_t) * v.size());
  return (int)v.size();
}

// ---------------- Ethereum validity on a hand-built DAG (ethereum_test.ml:44-77)
struct EthDag {
  std::vector<std::unique_ptr<Block>> blocks;
};
void* oracle_eth_dag_new(int root_height, int root_work) {
  auto* d = new EthDag();
  auto r = std::make_unique<Block>();
  r->value.height = root_height;
  r->value.work = root_work;
  r->value.miner = -1;
  r->has_pow = true;
  d->blocks.push_back(std::move(r));
  return d;
}
void oracle_eth_dag_free(void* d) { delete (EthDag*)d; }
// appends a block (always, like Dag.append) and returns its validity; *id = its index
int oracle_eth_dag_mine(void* dp, int parent, const int32_t* uncles, int n_uncles, int32_t* id) {
  auto* d = (EthDag*)dp;
  auto b = std::make_unique<Block>();
  Block* p = d->blocks[parent].get();
  b->parents.push_back(p);
  for (int i = 0; i < n_uncles; i++) b->parents.push_back(d->blocks[uncles[i]].get());
  b->value.height = p->value.height + 1;
  b->value.work = p->value.work + n_uncles + 1;
  b->value.miner = 42;
  b->has_pow = true;
  for (auto* q : b->parents) q->children_app.push_back(b.get());
  *id = (int32_t)d->blocks.size();
  Block* raw = b.get();
  d->blocks.push_back(std::move(b));
  return eth_validity(raw) ? 1 : 0;
}

// ---------------- ethereum_ssz policies / observation encoding
int oracle_eth_policy(int policy, const int32_t obs[10], const uint8_t* table, int dim) {
  EthObs o{obs[0], obs[1], obs[2], obs[3], obs[4], obs[5], obs[6], obs[7], obs[8], obs[9]};
  EthTable t;
  if (policy == ETH_POL_TABLE) {
    t.dim = dim;
    t.actions.assign(table, table + (size_t)dim * dim * 2);
  }
  return eth_policy(policy, o, &t);
}
void oracle_eth_obs_to_floats(const int32_t obs[10], int unit, double out[10]) {
  EthObs o{obs[0], obs[1], obs[2], obs[3], obs[4], obs[5], obs[6], obs[7], obs[8], obs[9]};
  eth_obs_to_floats(o, unit != 0, out);
}
void oracle_eth_obs_of_floats(const double in[10], int unit, int32_t out[10]) {
  EthObs o = eth_obs_of_floats(in, unit != 0);
  const int32_t v[10] = {o.public_height,  o.public_work,
                         o.private_height, o.private_work,
                         o.diff_height,    o.diff_work,
                         o.public_orphans, o.private_orphans_inclusive,
                         o.private_orphans_exclusive, o.event};
  memcpy(out, v, sizeof(v));
}

// ---------------- Ethereum gym env handle (engine.ml:97-273 for ethereum_ssz)
void* oracle_eth_gym_new(const cpr_config* c, int rng_mode, void* ocaml_rng, uint64_t episode) {
  try {
    return new GymEthereum(params_of(c), c->reward_scheme, rng_mode, (OcamlRandom*)ocaml_rng,
                           c->seed, episode);
  } catch (std::exception& e) {
    set_err(e.what());
    return nullptr;
  }
}
void oracle_eth_gym_free(void* g) { delete (GymEthereum*)g; }
int oracle_eth_gym_reset(void* g, double obs[10]) {
  try {
    ((GymEthereum*)g)->reset(obs);
    return 0;
  } catch (std::exception& e) {
    set_err(e.what());
    return -1;
  }
}
int oracle_eth_gym_obs_fields(void* g, int32_t out[10]) {
  double tmp[10];
  EthObs o = ((GymEthereum*)g)->observe_int();
  eth_obs_to_floats(o, false, tmp);
  for (int i = 0; i < 10; i++) out[i] = (int32_t)tmp[i];
  return 0;
}
// info_out: 12 doubles in engine.ml:226-237 order + head_height + head_miner + head_work
int oracle_eth_gym_step(void* g, int action, double obs[10], double* reward, int* done,
                        double info_out[15]) {
  try {
    bool d = false;
    StepInfo i;
    *reward = ((GymEthereum*)g)->step(action, obs, &d, &i);
    *done = d ? 1 : 0;
    if (info_out) {
      double v[15] = {i.step_reward_attacker,    i.step_reward_defender,
                      i.step_progress,           i.step_chain_time,
                      i.step_sim_time,           i.episode_reward_attacker,
                      i.episode_reward_defender, i.episode_progress,
                      i.episode_chain_time,      i.episode_sim_time,
                      (double)i.episode_n_steps, (double)i.episode_n_activations,
                      (double)i.head_height,     (double)i.head_miner,
                      (double)i.head_work};
      memcpy(info_out, v, sizeof(v));
    }
    return 0;
  } catch (std::exception& e) {
    set_err(e.what());
    return -1;
  }
}
uint32_t oracle_eth_gym_diag(void* g) { return ((GymEthereum*)g)->sim->diag; }

// the table of a CPR_ETH_POLICY_TABLE loop task (set per call by run_loop_episode)
static thread_local const EthTable* g_eth_table = nullptr;

int oracle_eth_two_agents_task(int rng_mode, void* rng, uint64_t seed, uint64_t episode,
                               double alpha, int scheme, int policy, int activations,
                               int64_t acts_out[2], double rewards_out[2], double* head_time,
                               double* head_progress, int32_t* head_height,
                               int32_t* head_work, uint32_t* diag) {
  try {
    EthLoopResult r;
    eth_two_agents_task(rng_mode, (OcamlRandom*)rng, seed, episode, alpha, scheme, policy,
                        activations, &r, g_eth_table);
    for (int i = 0; i < 2; i++) {
      acts_out[i] = r.activations[i];
      rewards_out[i] = r.rewards[i];
    }
    *head_time = r.head_time;
    *head_progress = r.head_progress;
    *head_height = r.head_height;
    *head_work = r.head_work;
    if (diag) *diag = r.diag;
    return 0;
  } catch (std::exception& e) {
    set_err(e.what());
    return -1;
  }
}

// ---------------- batch of full episodes (keyed stream), the CPU baseline workload
static int run_eth_gym_episode(const cpr_config* c, uint64_t ep, cpr_episode_record* rec) {
  const EthTable et = eth_table_of(c);
  GymEthereum g(params_of(c), c->reward_scheme, 1, nullptr, c->seed, ep);
  double obs[10];
  g.reset(obs);
  bool done = false;
  StepInfo info{};
  while (!done) {
    int a = eth_policy(c->policy, g.observe_int(), &et);
    g.step(a, obs, &done, &info);
  }
  rec->reward_attacker = info.episode_reward_attacker;
  rec->reward_defender = info.episode_reward_defender;
  rec->progress = info.episode_progress;
  rec->chain_time = info.episode_chain_time;
  rec->sim_time = info.episode_sim_time;
  rec->n_steps = info.episode_n_steps;
  rec->n_activations = info.episode_n_activations;
  rec->head_height = info.head_height;
  rec->head_miner = info.head_miner;
  rec->status = ((g.sim->diag & DIAG_TIE) ? (uint32_t)CPR_ST_TIE : 0u) |
                ((g.sim->diag & DIAG_OVERLAP) ? (uint32_t)CPR_ST_OVERLAP : 0u);
  rec->head_work = info.head_work;
  return 0;
}

static BkTable bk_table_of(const cpr_config* c) {
  BkTable t;
  if (c->protocol == CPR_PROTO_BK && c->policy == BKPOL_TABLE) {
    t.dim = c->policy_table_dim;
    t.k = c->k;
    t.actions.assign(c->policy_table, c->policy_table + bk_table_size(t.dim, t.k));
  }
  return t;
}

static int run_bk_gym_episode(const cpr_config* c, const BkTable* tab, uint64_t ep,
                              cpr_episode_record* rec) {
  GymBk g(params_of(c), c->k, c->reward_scheme, 1, nullptr, c->seed, ep);
  double obs[BK_OBS_LEN];
  g.reset(obs);
  bool done = false;
  StepInfo info{};
  while (!done) {
    int a = bk_policy(c->policy, g.observe_int(), c->k, tab);
    g.step(a, obs, &done, &info);
  }
  rec->reward_attacker = info.episode_reward_attacker;
  rec->reward_defender = info.episode_reward_defender;
  rec->progress = info.episode_progress;
  rec->chain_time = info.episode_chain_time;
  rec->sim_time = info.episode_sim_time;
  rec->n_steps = info.episode_n_steps;
  rec->n_activations = info.episode_n_activations;
  rec->head_height = info.head_height;
  rec->head_miner = info.head_miner;
  rec->status = 0;
  rec->head_work = 0;
  return 0;
}

// An episode in which the reference raises (List.for_all2 in summary dedup,
// Division_by_zero in n_choose_k, assert false / assert in tailstorm.ml) ends with status
// CPR_ST_REFERENCE_RAISES and zero outputs; one whose optimal quorum would brute-force past
// the budget (tailstorm.ml:418-507, the device's limit) with CPR_ST_CAPACITY. The device
// lane flags the same episodes (tests/native/ts_vs_oracle.cpp checks the step).
static void flagged_record(cpr_episode_record* rec, uint32_t status) {
  memset(rec, 0, sizeof(*rec));
  rec->head_miner = -1;
  rec->status = status;
}

static int run_ts_gym_episode(const cpr_config* c, uint64_t ep, cpr_episode_record* rec) {
  const TsTable tt = ts_table_of(c);
  GymTailstorm g(params_of(c), c->k, c->reward_scheme, c->subblock_selection, 1, nullptr,
                 c->seed, ep);
  double obs[TS_OBS_LEN];
  bool done = false;
  StepInfo info{};
  try {
    g.reset(obs);
    while (!done) {
      int a = ts_policy(c->policy, g.observe_int(), c->k, &tt);
      g.step(a, obs, &done, &info);
    }
  } catch (BudgetExceeded&) {
    flagged_record(rec, CPR_ST_CAPACITY);
    return 0;
  } catch (std::exception&) {
    flagged_record(rec, CPR_ST_REFERENCE_RAISES);
    return 0;
  }
  rec->reward_attacker = info.episode_reward_attacker;
  rec->reward_defender = info.episode_reward_defender;
  rec->progress = info.episode_progress;
  rec->chain_time = info.episode_chain_time;
  rec->sim_time = info.episode_sim_time;
  rec->n_steps = info.episode_n_steps;
  rec->n_activations = info.episode_n_activations;
  rec->head_height = info.head_height;
  rec->head_miner = info.head_miner;
  rec->status = 0;
  rec->head_work = 0;
  return 0;
}

static int run_gym_episode(const cpr_config* c, const TablePolicy* tab, uint64_t ep,
                           cpr_episode_record* rec) {
  if (c->protocol == CPR_PROTO_ETHEREUM) return run_eth_gym_episode(c, ep, rec);
  if (c->protocol == CPR_PROTO_TAILSTORM) return run_ts_gym_episode(c, ep, rec);
  if (c->protocol == CPR_PROTO_BK) {
    BkTable bt = bk_table_of(c);
    return run_bk_gym_episode(c, &bt, ep, rec);
  }
  GymNakamoto g(params_of(c), 1, nullptr, c->seed, ep);
  double obs[4];
  g.reset(obs);
  bool done = false;
  StepInfo info{};
  while (!done) {
    int a = nak_policy(c->policy, g.observe_int(), tab);
    g.step(a, obs, &done, &info);
  }
  rec->reward_attacker = info.episode_reward_attacker;
  rec->reward_defender = info.episode_reward_defender;
  rec->progress = info.episode_progress;
  rec->chain_time = info.episode_chain_time;
  rec->sim_time = info.episode_sim_time;
  rec->n_steps = info.episode_n_steps;
  rec->n_activations = info.episode_n_activations;
  rec->head_height = info.head_height;
  rec->head_miner = info.head_miner;
  rec->status = ((g.sim->diag & DIAG_TIE) ? (uint32_t)CPR_ST_TIE : 0u) |
                ((g.sim->diag & DIAG_OVERLAP) ? (uint32_t)CPR_ST_OVERLAP : 0u);
  rec->head_work = 0;
  return 0;
}

// Networks of the B_k / Tailstorm loop tasks. 0: two_agents(alpha); 1: symmetric clique of
// n_nodes with exponential(prop_ev) delays (cpr_protocols.ml:200-210,478-485); 2: models.ml:3-28
// honest_clique (compute i + 1, uniform lo .. hi delays)
static Network loop_net(int net_kind, int n_nodes, double alpha, double activation_delay,
                        double prop_ev, double lo, double hi) {
  if (net_kind == 0) return Network::two_agents(activation_delay, alpha);
  Network net;
  net.flooding = false;
  net.activation_delay = activation_delay;
  net.nodes.resize(n_nodes);
  for (int i = 0; i < n_nodes; ++i) {
    net.nodes[i].compute = net_kind == 2 ? (double)(i + 1) : 1. / (double)n_nodes;
    for (int j = 0; j < n_nodes - 1; ++j)
      net.nodes[i].links.push_back(net_kind == 2 ? Link{j >= i ? j + 1 : j, D_UNIFORM, lo, hi}
                                                 : Link{j >= i ? j + 1 : j, D_EXP, prop_ev, 0.0});
  }
  return net;
}

// Per-node outputs of a loop task (csv_runner.ml:74-79 `activations` / `reward` columns):
// run_loop_episode copies its per-node vectors here when a caller set the sink
// (oracle_node_outputs); head_miner -2 = not reported
struct NodeSink {
  int64_t* acts = nullptr;
  double* rews = nullptr;
  int32_t* head_miner = nullptr;
  int n = 0;
};
static thread_local NodeSink g_sink;

static void sink_nodes(const int64_t* a, const double* r, int n, int32_t hm) {
  if (!g_sink.acts) return;
  if (n != g_sink.n) throw std::runtime_error("node outputs: node count mismatch");
  for (int i = 0; i < n; ++i) {
    g_sink.acts[i] = a[i];
    g_sink.rews[i] = r[i];
  }
  *g_sink.head_miner = hm;
}

static TablePolicy table_of(const cpr_config* c);

// Nakamoto / Ethereum Simulator.loop task on the exponential-delay clique
// (cpr_protocols.ml:200-210,478-485): node 0 runs nakamoto_ssz / ethereum_ssz with the
// policy (or table), `defenders` honest nodes, equal compute, exponential(propagation_delay)
// links keyed by share window (kw, off, dest), keyed stream
static int attack_clique_task(const cpr_config* c, uint64_t ep, cpr_episode_record* rec) {
  try {
    const bool eth = c->protocol == CPR_PROTO_ETHEREUM;
    const int n = c->defenders + 1;
    const Network net = loop_net(1, n, 0.0, c->activation_delay, c->propagation_delay, 0.0, 0.0);
    std::unique_ptr<SimRng> rng(new KeyedSimRng(c->seed, ep, net));
    rng = trace_wrap(std::move(rng), net, false);
    Sim sim(net, rng.get());
    if (eth) {
      sim.proto = 1;
      sim.eth_scheme = c->reward_scheme;
    }
    const EthTable et = eth_table_of(c);
    const TablePolicy nt = table_of(c);
    std::vector<std::unique_ptr<NodeImpl>> nodes;
    NakSszAttackerNode* na = nullptr;
    EthSszAttackerNode* ea = nullptr;
    if (eth) {
      ea = new EthSszAttackerNode();
      ea->policy = c->policy;
      ea->table = &et;
      nodes.emplace_back(ea);
    } else {
      na = new NakSszAttackerNode();
      na->policy = c->policy;
      na->table = c->policy == POL_TABLE ? &nt : nullptr;
      nodes.emplace_back(na);
    }
    for (int i = 1; i < n; ++i) {
      if (eth)
        nodes.emplace_back(new EthHonest());
      else
        nodes.emplace_back(new NakHonest());
    }
    sim.init(std::move(nodes));
    Block* root = sim.roots.back();
    if (eth) {
      ea->agent.sim = &sim;
      ea->agent.my_id = 0;
      ea->agent.init(root);
      for (int i = 1; i < n; ++i) static_cast<EthHonest*>(sim.nodes[i].get())->state = root;
    } else {
      na->agent.sim = &sim;
      na->agent.my_id = 0;
      na->agent.init(root);
      for (int i = 1; i < n; ++i) static_cast<NakHonest*>(sim.nodes[i].get())->state = root;
    }
    sim.loop((int)c->activations);
    Block* h = sim.head();
    std::vector<int64_t> a(n);
    std::vector<double> rw(n);
    for (int i = 0; i < n; ++i) {
      a[i] = sim.activations[i];
      rw[i] = h->rewards[i];
    }
    sink_nodes(a.data(), rw.data(), n, eth ? -2 : h->value.miner);
    rec->reward_attacker = rw[0];
    rec->reward_defender = 0.0;
    rec->n_activations = 0;
    for (int i = 1; i < n; ++i) rec->reward_defender += rw[i];
    for (int i = 0; i < n; ++i) rec->n_activations += a[i];
    rec->progress = eth ? sim.progress(h) : (double)h->value.height;
    rec->chain_time = Sim::timestamp(h);
    rec->sim_time = 0.0;
    rec->n_steps = 0;
    rec->head_height = h->value.height;
    rec->head_miner = -1;
    rec->status = 0;
    rec->head_work = eth ? h->value.work : 0;
    return 0;
  } catch (std::exception& e) {
    set_err(e.what());
    return -1;
  }
}

static int run_loop_episode(const cpr_config* c, uint64_t ep, cpr_episode_record* rec) {
  int64_t acts[2];
  double rew[2], ht, hp;
  int32_t hh;
  uint32_t diag = 0;
  if (c->network == CPR_NET_HONEST_CLIQUE &&
      (c->protocol == CPR_PROTO_NAKAMOTO || c->protocol == CPR_PROTO_ETHEREUM)) {
    const int n = c->defenders;
    const bool dflt = std::isnan(c->delay_lo) && std::isnan(c->delay_hi);  // NaN: models.ml default
    std::vector<int64_t> a(n);
    std::vector<double> r(n);
    double ht, hp;
    int32_t hh, hm, hw;
    if (oracle_clique_task(c->protocol == CPR_PROTO_ETHEREUM ? 1 : 0, 1, nullptr, c->seed, ep, n,
                           c->activation_delay, dflt ? 0.5 : c->delay_lo,
                           dflt ? 1.5 : c->delay_hi, c->reward_scheme, (int)c->activations,
                           a.data(), r.data(), &ht, &hp, &hh, &hm, &hw) != 0)
      return -1;
    sink_nodes(a.data(), r.data(), n, c->protocol == CPR_PROTO_ETHEREUM ? -2 : hm);
    rec->reward_attacker = r[0];
    rec->reward_defender = 0.0;
    rec->n_activations = 0;
    for (int i = 1; i < n; ++i) rec->reward_defender += r[i];
    for (int i = 0; i < n; ++i) rec->n_activations += a[i];
    rec->progress = hp;
    rec->chain_time = ht;
    rec->sim_time = 0.0;
    rec->n_steps = 0;
    rec->head_height = hh;
    rec->head_miner = -1;
    rec->status = 0;
    rec->head_work = c->protocol == CPR_PROTO_ETHEREUM ? hw : 0;
    return 0;
  }
  if (c->network == CPR_NET_HONEST_CLIQUE &&
      (c->protocol == CPR_PROTO_BK || c->protocol == CPR_PROTO_TAILSTORM)) {
    // every node honest (policy ignored), keyed stream
    const bool dflt = std::isnan(c->delay_lo) && std::isnan(c->delay_hi);  // NaN: models.ml default
    const Network net = loop_net(2, c->defenders, 0.0, c->activation_delay, 0.0,
                                 dflt ? 0.5 : c->delay_lo, dflt ? 1.5 : c->delay_hi);
    std::vector<double> rw;
    std::vector<int64_t> ac;
    if (c->protocol == CPR_PROTO_BK) {
      BkLoopResult r;
      bk_loop_task(net, 1, nullptr, c->seed, ep, c->k, c->reward_scheme, -1, nullptr,
                   (int)c->activations, &r);
      rw = r.rewards;
      ac.assign(r.activations.begin(), r.activations.end());
      rec->progress = r.head_progress;
      rec->chain_time = r.head_time;
      rec->head_height = r.head_height;
      rec->head_miner = r.head_signer;
      sink_nodes(ac.data(), rw.data(), (int)rw.size(), r.head_signer);
    } else {
      TsLoopResult r;
      try {
        ts_loop_task(net, 1, nullptr, c->seed, ep, c->k, c->reward_scheme,
                     c->subblock_selection, -1, (int)c->activations, &r);
      } catch (BudgetExceeded&) {
        flagged_record(rec, CPR_ST_CAPACITY);
        return 0;
      } catch (std::exception&) {
        flagged_record(rec, CPR_ST_REFERENCE_RAISES);
        return 0;
      }
      rw = r.rewards;
      ac.assign(r.activations.begin(), r.activations.end());
      rec->progress = r.head_progress;
      rec->chain_time = r.head_time;
      rec->head_height = r.head_height;
      rec->head_miner = -1;
      sink_nodes(ac.data(), rw.data(), (int)rw.size(), -1);
    }
    rec->reward_attacker = rw[0];
    rec->reward_defender = 0.0;
    rec->n_activations = 0;
    for (size_t i = 1; i < rw.size(); ++i) rec->reward_defender += rw[i];
    for (int64_t a : ac) rec->n_activations += a;
    rec->sim_time = 0.0;
    rec->n_steps = 0;
    rec->status = 0;
    rec->head_work = 0;
    return 0;
  }
  if (c->network == CPR_NET_SELFISH_MINING && c->protocol == CPR_PROTO_NAKAMOTO) {
    const int n = c->defenders + 1;
    std::vector<int64_t> a(n);
    std::vector<double> r(n);
    int32_t hm = -1;
    if (oracle_sm_task(1, nullptr, c->seed, ep, c->alpha, c->gamma, c->defenders,
                       c->propagation_delay > 0 ? c->propagation_delay : 1e-9, c->policy,
                       (int)c->activations, a.data(), r.data(), &ht, &hp, &hh, &hm, &diag) != 0)
      return -1;
    sink_nodes(a.data(), r.data(), n, hm);
    rec->reward_attacker = r[0];
    rec->reward_defender = 0.0;
    rec->n_activations = 0;
    for (int i = 1; i < n; ++i) rec->reward_defender += r[i];
    for (int i = 0; i < n; ++i) rec->n_activations += a[i];
    rec->progress = hp;
    rec->chain_time = ht;
    rec->sim_time = 0.0;
    rec->n_steps = 0;
    rec->head_height = hh;
    rec->head_miner = -1;  // as every loop-mode record (oracle_sm_task reports the miner)
    (void)hm;
    rec->status = 0;
    rec->head_work = 0;
    return 0;
  }
  if (c->network == CPR_NET_EXP_CLIQUE &&
      (c->protocol == CPR_PROTO_NAKAMOTO || c->protocol == CPR_PROTO_ETHEREUM))
    return attack_clique_task(c, ep, rec);
  if (c->network == CPR_NET_EXP_CLIQUE &&
      (c->protocol == CPR_PROTO_BK || c->protocol == CPR_PROTO_TAILSTORM)) {
    // symmetric clique, exponential(propagation_delay) links, node 0 runs the policy
    // (cpr_protocols.ml:200-210,478-485), keyed stream
    const Network net = loop_net(1, c->defenders + 1, 0.0, c->activation_delay,
                                 c->propagation_delay, 0.0, 0.0);
    std::vector<double> rw;
    std::vector<int64_t> ac;
    if (c->protocol == CPR_PROTO_BK) {
      BkTable bt = bk_table_of(c);
      BkLoopResult r;
      bk_loop_task(net, 1, nullptr, c->seed, ep, c->k, c->reward_scheme, c->policy, &bt,
                   (int)c->activations, &r);
      rw = r.rewards;
      ac.assign(r.activations.begin(), r.activations.end());
      rec->progress = r.head_progress;
      rec->chain_time = r.head_time;
      rec->head_height = r.head_height;
      rec->head_miner = r.head_signer;
      sink_nodes(ac.data(), rw.data(), (int)rw.size(), r.head_signer);
    } else {
      TsLoopResult r;
      try {
        const TsTable tt = ts_table_of(c);
        ts_loop_task(net, 1, nullptr, c->seed, ep, c->k, c->reward_scheme,
                     c->subblock_selection, c->policy, (int)c->activations, &r, &tt);
      } catch (BudgetExceeded&) {
        flagged_record(rec, CPR_ST_CAPACITY);
        return 0;
      } catch (std::exception&) {
        flagged_record(rec, CPR_ST_REFERENCE_RAISES);
        return 0;
      }
      rw = r.rewards;
      ac.assign(r.activations.begin(), r.activations.end());
      rec->progress = r.head_progress;
      rec->chain_time = r.head_time;
      rec->head_height = r.head_height;
      rec->head_miner = -1;
      sink_nodes(ac.data(), rw.data(), (int)rw.size(), -1);
    }
    rec->reward_attacker = rw[0];
    rec->reward_defender = 0.0;
    rec->n_activations = 0;
    for (size_t i = 1; i < rw.size(); ++i) rec->reward_defender += rw[i];
    for (int64_t a : ac) rec->n_activations += a;
    rec->sim_time = 0.0;
    rec->n_steps = 0;
    rec->status = 0;
    rec->head_work = 0;
    return 0;
  }
  if (c->network != CPR_NET_TWO_AGENTS) {
    set_err("oracle loop mode: two-agents network, selfish-mining network (Nakamoto) or "
            "honest clique only");
    return -2;
  }
  if (c->protocol == CPR_PROTO_TAILSTORM) {
    TsLoopResult r;
    try {
      const TsTable tt = ts_table_of(c);
      ts_loop_task(Network::two_agents(c->activation_delay, c->alpha), 1, nullptr, c->seed, ep,
                   c->k, c->reward_scheme, c->subblock_selection, c->policy,
                   (int)c->activations, &r, &tt);
    } catch (BudgetExceeded&) {
      flagged_record(rec, CPR_ST_CAPACITY);
      return 0;
    } catch (std::exception&) {
      flagged_record(rec, CPR_ST_REFERENCE_RAISES);
      return 0;
    }
    {
      const int64_t a2[2] = {r.activations[0], r.activations[1]};
      sink_nodes(a2, r.rewards.data(), 2, -1);
    }
    rec->reward_attacker = r.rewards[0];
    rec->reward_defender = r.rewards[1];
    rec->progress = r.head_progress;
    rec->chain_time = r.head_time;
    rec->sim_time = 0.0;
    rec->n_steps = 0;
    rec->n_activations = r.activations[0] + r.activations[1];
    rec->head_height = r.head_height;
    rec->head_miner = -1;
    rec->status = 0;
    rec->head_work = 0;
    return 0;
  }
  if (c->protocol == CPR_PROTO_BK) {
    BkTable bt = bk_table_of(c);
    BkLoopResult r;
    bk_loop_task(Network::two_agents(c->activation_delay, c->alpha), 1, nullptr, c->seed, ep,
                 c->k, c->reward_scheme, c->policy, &bt, (int)c->activations, &r);
    {
      const int64_t a2[2] = {r.activations[0], r.activations[1]};
      sink_nodes(a2, r.rewards.data(), 2, r.head_signer);
    }
    rec->reward_attacker = r.rewards[0];
    rec->reward_defender = r.rewards[1];
    rec->progress = r.head_progress;
    rec->chain_time = r.head_time;
    rec->sim_time = 0.0;
    rec->n_steps = 0;
    rec->n_activations = r.activations[0] + r.activations[1];
    rec->head_height = r.head_height;
    rec->head_miner = r.head_signer;
    rec->status = 0;
    rec->head_work = 0;
    return 0;
  }
  if (c->protocol == CPR_PROTO_ETHEREUM) {
    int32_t hw = 0;
    const EthTable et = eth_table_of(c);
    g_eth_table = &et;
    const int rc = oracle_eth_two_agents_task(1, nullptr, c->seed, ep, c->alpha,
                                              c->reward_scheme, c->policy, (int)c->activations,
                                              acts, rew, &ht, &hp, &hh, &hw, &diag);
    g_eth_table = nullptr;
    if (rc != 0) return -1;
    sink_nodes(acts, rew, 2, -2);
    rec->reward_attacker = rew[0];
    rec->reward_defender = rew[1];
    rec->progress = hp;
    rec->chain_time = ht;
    rec->sim_time = 0.0;
    rec->n_steps = 0;
    rec->n_activations = acts[0] + acts[1];
    rec->head_height = hh;
    rec->head_miner = -1;
    rec->status = 0;
    rec->head_work = hw;
    return 0;
  }
  if (oracle_two_agents_task(1, nullptr, c->seed, ep, c->alpha, c->policy,
                             (int)c->activations, acts, rew, &ht, &hp, &hh, &diag) != 0)
    return -1;
  sink_nodes(acts, rew, 2, -2);
  rec->reward_attacker = rew[0];
  rec->reward_defender = rew[1];
  rec->progress = hp;
  rec->chain_time = ht;
  rec->sim_time = 0.0;
  rec->n_steps = 0;
  rec->n_activations = acts[0] + acts[1];
  rec->head_height = hh;
  rec->head_miner = -1;
  rec->status = 0;
  rec->head_work = 0;
  return 0;
}

// ---------------- B_k (bk.ml, bk_ssz.ml)
int oracle_bk_policy(int policy, const int32_t obs[8], int k, const uint8_t* table, int dim) {
  BkTable t;
  if (policy == BKPOL_TABLE) {
    t.dim = dim;
    t.k = k;
    t.actions.assign(table, table + bk_table_size(dim, k));
  }
  BkObs o{obs[0], obs[1], obs[2], obs[3], obs[4], obs[5], obs[6], obs[7]};
  return bk_policy(policy, o, k, &t);
}
void oracle_bk_obs_to_floats(const int32_t obs[8], int unit, int k, double out[8]) {
  BkObs o{obs[0], obs[1], obs[2], obs[3], obs[4], obs[5], obs[6], obs[7]};
  bk_obs_to_floats(o, unit != 0, k, out);
}
void oracle_bk_obs_of_floats(const double in[8], int unit, int k, int32_t out[8]) {
  BkObs o = bk_obs_of_floats(in, unit != 0, k);
  const int32_t v[8] = {o.public_blocks,           o.private_blocks, o.diff_blocks,
                        o.public_votes,            o.private_votes_inclusive,
                        o.private_votes_exclusive, o.lead,           o.event};
  memcpy(out, v, sizeof(v));
}
void oracle_bk_obs_range(int unit, double low[8], double high[8]) {
  bk_obs_range(unit != 0, low, high);
}
void* oracle_bk_gym_new(const cpr_config* c, int rng_mode, void* ocaml_rng, uint64_t episode) {
  try {
    return new GymBk(params_of(c), c->k, c->reward_scheme, rng_mode, (OcamlRandom*)ocaml_rng,
                     c->seed, episode);
  } catch (std::exception& e) {
    set_err(e.what());
    return nullptr;
  }
}
void oracle_bk_gym_free(void* g) { delete (GymBk*)g; }
int oracle_bk_gym_reset(void* g, double obs[8]) {
  try {
    ((GymBk*)g)->reset(obs);
    return 0;
  } catch (std::exception& e) {
    set_err(e.what());
    return -1;
  }
}
int oracle_bk_gym_obs_fields(void* g, int32_t out[8]) {
  BkObs o = ((GymBk*)g)->observe_int();
  const int32_t v[8] = {o.public_blocks,           o.private_blocks, o.diff_blocks,
                        o.public_votes,            o.private_votes_inclusive,
                        o.private_votes_exclusive, o.lead,           o.event};
  memcpy(out, v, sizeof(v));
  return 0;
}
// info_out: 12 doubles in engine.ml:226-237 order + head_height + head signer + n_vertices
int oracle_bk_gym_step(void* g, int action, double obs[8], double* reward, int* done,
                       double info_out[15]) {
  try {
    bool d = false;
    StepInfo i;
    GymBk* e = (GymBk*)g;
    *reward = e->step(action, obs, &d, &i);
    *done = d ? 1 : 0;
    if (info_out) {
      double v[15] = {i.step_reward_attacker,    i.step_reward_defender,
                      i.step_progress,           i.step_chain_time,
                      i.step_sim_time,           i.episode_reward_attacker,
                      i.episode_reward_defender, i.episode_progress,
                      i.episode_chain_time,      i.episode_sim_time,
                      (double)i.episode_n_steps, (double)i.episode_n_activations,
                      (double)i.head_height,     (double)i.head_miner,
                      (double)e->sim->dag.size()};
      memcpy(info_out, v, sizeof(v));
    }
    return 0;
  } catch (std::exception& e) {
    set_err(e.what());
    return -1;
  }
}
// Simulator.loop task for B_k. net_kind 0: two_agents(alpha); 1: symmetric_clique of n_nodes
// with exponential(prop_ev) propagation delays (cpr_protocols.ml:200-210,478-485).
// policy < 0: node 0 honest. rewards_out / acts_out: n_nodes entries.
int oracle_bk_loop(int net_kind, int n_nodes, double alpha, double activation_delay,
                   double prop_ev, int rng_mode, void* rng, uint64_t seed, uint64_t episode,
                   int k, int scheme, int policy, int activations, double* rewards_out,
                   int64_t* acts_out, double* head_time, double* head_progress,
                   int32_t* head_height, int32_t* head_signer, int64_t* n_vertices) {
  try {
    const Network net = loop_net(net_kind, n_nodes, alpha, activation_delay, prop_ev, 0.5, 1.5);
    BkTable t;
    BkLoopResult r;
    bk_loop_task(net, rng_mode, (OcamlRandom*)rng, seed, episode, k, scheme, policy, &t,
                 activations, &r);
    for (size_t i = 0; i < r.rewards.size(); ++i) {
      rewards_out[i] = r.rewards[i];
      acts_out[i] = r.activations[i];
    }
    *head_time = r.head_time;
    *head_progress = r.head_progress;
    *head_height = r.head_height;
    *head_signer = r.head_signer;
    *n_vertices = r.n_vertices;
    return 0;
  } catch (std::exception& e) {
    set_err(e.what());
    return -1;
  }
}

// ---------------- Tailstorm (tailstorm.ml, tailstorm_ssz.ml)
int oracle_ts_policy(int policy, const int32_t obs[10], int k, const uint8_t* table, int dim) {
  TsObs o{obs[0], obs[1], obs[2], obs[3], obs[4], obs[5], obs[6], obs[7], obs[8], obs[9]};
  TsTable t;
  if (policy == TS_POL_TABLE) {
    t.dim = dim;
    const size_t K1 = (size_t)k + 1;
    t.actions.assign(table, table + (size_t)dim * dim * K1 * K1 * 3);
  }
  return ts_policy(policy, o, k, &t);
}
void oracle_ts_obs_to_floats(const int32_t obs[10], int unit, int k, double out[10]) {
  TsObs o{obs[0], obs[1], obs[2], obs[3], obs[4], obs[5], obs[6], obs[7], obs[8], obs[9]};
  ts_obs_to_floats(o, unit != 0, k, out);
}
void oracle_ts_obs_of_floats(const double in[10], int unit, int k, int32_t out[10]) {
  TsObs o = ts_obs_of_floats(in, unit != 0, k);
  const int32_t v[10] = {o.public_blocks,           o.private_blocks,
                         o.diff_blocks,             o.public_votes,
                         o.private_votes_inclusive, o.private_votes_exclusive,
                         o.public_depth,            o.private_depth_inclusive,
                         o.private_depth_exclusive, o.event};
  memcpy(out, v, sizeof(v));
}
int64_t oracle_n_choose_k(int64_t n, int64_t k) {
  try {
    return ocaml_n_choose_k(n, k);
  } catch (std::exception& e) {
    set_err(e.what());
    return -1;
  }
}
void* oracle_ts_gym_new(const cpr_config* c, int rng_mode, void* ocaml_rng, uint64_t episode) {
  try {
    return new GymTailstorm(params_of(c), c->k, c->reward_scheme, c->subblock_selection,
                            rng_mode, (OcamlRandom*)ocaml_rng, c->seed, episode);
  } catch (std::exception& e) {
    set_err(e.what());
    return nullptr;
  }
}
void oracle_ts_gym_free(void* g) { delete (GymTailstorm*)g; }
int oracle_ts_gym_reset(void* g, double obs[10]) {
  try {
    ((GymTailstorm*)g)->reset(obs);
    return 0;
  } catch (std::exception& e) {
    set_err(e.what());
    return -1;
  }
}
int oracle_ts_gym_obs_fields(void* g, int32_t out[10]) {
  TsObs o = ((GymTailstorm*)g)->observe_int();
  const int32_t v[10] = {o.public_blocks,           o.private_blocks,
                         o.diff_blocks,             o.public_votes,
                         o.private_votes_inclusive, o.private_votes_exclusive,
                         o.public_depth,            o.private_depth_inclusive,
                         o.private_depth_exclusive, o.event};
  memcpy(out, v, sizeof(v));
  return 0;
}
int oracle_ts_gym_step(void* g, int action, double obs[10], double* reward, int* done,
                       double info_out[15]) {
  try {
    bool d = false;
    StepInfo i;
    GymTailstorm* e = (GymTailstorm*)g;
    *reward = e->step(action, obs, &d, &i);
    *done = d ? 1 : 0;
    if (info_out) {
      double v[15] = {i.step_reward_attacker,    i.step_reward_defender,
                      i.step_progress,           i.step_chain_time,
                      i.step_sim_time,           i.episode_reward_attacker,
                      i.episode_reward_defender, i.episode_progress,
                      i.episode_chain_time,      i.episode_sim_time,
                      (double)i.episode_n_steps, (double)i.episode_n_activations,
                      (double)i.head_height,     (double)i.head_miner,
                      (double)e->sim->dag.size()};
      memcpy(info_out, v, sizeof(v));
    }
    return 0;
  } catch (std::exception& e) {
    set_err(e.what());
    return -1;
  }
}
// Simulator.loop task for Tailstorm. net_kind 0: two_agents(alpha); 1: symmetric_clique of
// n_nodes with exponential(prop_ev) delays. policy < 0: node 0 honest.
int oracle_ts_loop(int net_kind, int n_nodes, double alpha, double activation_delay,
                   double prop_ev, int rng_mode, void* rng, uint64_t seed, uint64_t episode,
                   int k, int scheme, int selection, int policy, int activations,
                   double* rewards_out, int64_t* acts_out, double* head_time,
                   double* head_progress, int32_t* head_height, int64_t* n_vertices) {
  try {
    const Network net = loop_net(net_kind, n_nodes, alpha, activation_delay, prop_ev, 0.5, 1.5);
    TsLoopResult r;
    ts_loop_task(net, rng_mode, (OcamlRandom*)rng, seed, episode, k, scheme, selection, policy,
                 activations, &r);
    for (size_t i = 0; i < r.rewards.size(); ++i) {
      rewards_out[i] = r.rewards[i];
      acts_out[i] = r.activations[i];
    }
    *head_time = r.head_time;
    *head_progress = r.head_progress;
    *head_height = r.head_height;
    *n_vertices = r.n_vertices;
    return 0;
  } catch (std::exception& e) {
    set_err(e.what());
    return -1;
  }
}

// ---------------- activation/delay traces (cpr_trace)
// Record: run episodes [first, first + n) of config c in order on this thread with every
// draw logged by keyed coordinate. rng_mode 1 draws from the keyed stream; rng_mode 0
// from the OCaml Random state `rng`, carried from episode to episode like one Parany
// worker (the reference's own stream). Returns a handle (NULL on error).
struct TraceSet {
  std::vector<TraceBuf> eps;
};

static TablePolicy table_of(const cpr_config* c) {
  TablePolicy tab;
  if (c->protocol == CPR_PROTO_NAKAMOTO && c->policy == POL_TABLE) {
    tab.dim = c->policy_table_dim;
    tab.actions.assign(c->policy_table, c->policy_table + tab.dim * tab.dim * 2);
  }
  return tab;
}

static int run_one(const cpr_config* c, const TablePolicy* tab, uint64_t ep,
                   cpr_episode_record* rec) {
  return c->mode == CPR_MODE_GYM ? run_gym_episode(c, tab, ep, rec) : run_loop_episode(c, ep, rec);
}

void* oracle_trace_record(const cpr_config* c, int rng_mode, void* rng, uint64_t first,
                          int64_t n, cpr_episode_record* out) {
  auto* ts = new TraceSet();
  ts->eps.resize((size_t)n);
  const TablePolicy tab = table_of(c);
  int rc = 0;
  try {
    for (int64_t i = 0; i < n && rc == 0; i++) {
      g_trace.mode = TRACE_RECORD;
      g_trace.buf = &ts->eps[(size_t)i];
      g_trace.ocaml = rng_mode == 0 ? (OcamlRandom*)rng : nullptr;
      rc = run_one(c, &tab, first + (uint64_t)i, &out[i]);
    }
  } catch (std::exception& e) {
    set_err(e.what());
    rc = -1;
  }
  g_trace = TraceHook();
  if (rc != 0) {
    delete ts;
    return nullptr;
  }
  return ts;
}

// totals: [0] activations, [1] pow hashes, [2] link delays over all episodes
void oracle_trace_sizes(void* h, int64_t out[3]) {
  const TraceSet* ts = (const TraceSet*)h;
  out[0] = out[1] = out[2] = 0;
  for (const TraceBuf& b : ts->eps) {
    out[0] += (int64_t)b.delay.size();
    out[1] += (int64_t)b.pow.size();
    out[2] += (int64_t)b.link.size();
  }
}

// CSR arrays of cpr_trace; activation arrays have one entry per act_delay draw (the last
// clock of an episode is scheduled but never fires: its miner entry is 0)
void oracle_trace_fill(void* h, int64_t* act_off, int32_t* miner, double* delay, int64_t* pow_off,
                       int32_t* pow, int64_t* link_off, uint64_t* key, double* ldelay) {
  const TraceSet* ts = (const TraceSet*)h;
  int64_t a = 0, p = 0, l = 0;
  act_off[0] = pow_off[0] = link_off[0] = 0;
  for (size_t e = 0; e < ts->eps.size(); e++) {
    const TraceBuf& b = ts->eps[e];
    for (size_t j = 0; j < b.delay.size(); j++, a++) {
      delay[a] = b.delay[j];
      miner[a] = j < b.miner.size() ? b.miner[j] : 0;
    }
    for (size_t j = 0; j < b.pow.size(); j++) pow[p++] = b.pow[j];
    for (const auto& kv : b.link) {
      key[l] = kv.first;
      ldelay[l++] = kv.second;
    }
    act_off[e + 1] = a;
    pow_off[e + 1] = p;
    link_off[e + 1] = l;
  }
}

void oracle_trace_free(void* h) { delete (TraceSet*)h; }

// Replay: trace episode e drives record out[e]; out[e].status gets CPR_ST_TRACE_MISS when
// the episode needed a draw the trace lacks
int oracle_trace_replay(const cpr_config* c, const cpr_trace* t, cpr_episode_record* out) {
  const TablePolicy tab = table_of(c);
  int rc = 0;
  try {
    for (int64_t e = 0; e < t->n_episodes && rc == 0; e++) {
      TraceBuf b;
      for (int64_t i = t->act_offset[e]; i < t->act_offset[e + 1]; i++) {
        b.miner.push_back(t->act_miner[i]);
        b.delay.push_back(t->act_delay[i]);
      }
      for (int64_t i = t->pow_offset[e]; i < t->pow_offset[e + 1]; i++)
        b.pow.push_back(t->pow_hash[i]);
      for (int64_t i = t->link_offset[e]; i < t->link_offset[e + 1]; i++)
        b.link[t->link_key[i]] = t->link_delay[i];
      g_trace.mode = TRACE_REPLAY;
      g_trace.buf = &b;
      g_trace.ocaml = nullptr;
      rc = run_one(c, &tab, (uint64_t)e, &out[e]);
      if (b.miss) out[e].status |= CPR_ST_TRACE_MISS;
    }
  } catch (std::exception& e) {
    set_err(e.what());
    rc = -1;
  }
  g_trace = TraceHook();
  return rc;
}

// Per-node outputs of loop tasks (cpr_node_outputs' oracle): keyed episodes [first, first+n)
// or, with t != NULL, trace episodes; rows of n_nodes; head_miner -2 where the task does
// not report it
int oracle_node_outputs(const cpr_config* c, uint64_t first, int64_t n, const cpr_trace* t,
                        int n_nodes, cpr_episode_record* out, int64_t* acts, double* rews,
                        int32_t* head_miner) {
  if (c->mode != CPR_MODE_LOOP) {
    set_err("oracle node outputs: loop mode only");
    return -2;
  }
  if (t) n = t->n_episodes;
  int rc = 0;
  try {
    for (int64_t e = 0; e < n && rc == 0; e++) {
      g_sink.acts = acts + e * n_nodes;
      g_sink.rews = rews + e * n_nodes;
      g_sink.head_miner = head_miner + e;
      g_sink.n = n_nodes;
      head_miner[e] = -2;
      for (int i = 0; i < n_nodes; ++i) {
        g_sink.acts[i] = 0;
        g_sink.rews[i] = 0.0;
      }
      if (t) {
        cpr_trace one = *t;  // episode e of the trace as a one-episode trace
        int64_t offs[3][2] = {{0, t->act_offset[e + 1] - t->act_offset[e]},
                              {0, t->pow_offset[e + 1] - t->pow_offset[e]},
                              {0, t->link_offset[e + 1] - t->link_offset[e]}};
        one.n_episodes = 1;
        one.act_offset = offs[0];
        one.pow_offset = offs[1];
        one.link_offset = offs[2];
        one.act_miner = t->act_miner + t->act_offset[e];
        one.act_delay = t->act_delay + t->act_offset[e];
        one.pow_hash = t->pow_hash + t->pow_offset[e];
        one.link_key = t->link_key + t->link_offset[e];
        one.link_delay = t->link_delay + t->link_offset[e];
        rc = oracle_trace_replay(c, &one, &out[e]);
      } else {
        rc = run_loop_episode(c, first + (uint64_t)e, &out[e]);
      }
    }
  } catch (std::exception& ex) {
    set_err(ex.what());
    rc = -1;
  }
  g_sink = NodeSink();
  return rc;
}

// threads: number of worker threads (episode-parallel, like Parany workers)
int oracle_run_episodes(const cpr_config* c, uint64_t first, int64_t n, cpr_episode_record* out,
                        int threads) {
  TablePolicy tab;
  if (c->policy == POL_TABLE) {
    tab.dim = c->policy_table_dim;
    tab.actions.assign(c->policy_table, c->policy_table + tab.dim * tab.dim * 2);
  }
  if (threads < 1) threads = 1;
  std::vector<int> rc(threads, 0);
  std::vector<std::string> errs(threads);
  auto work = [&](int t) {
    try {
      for (int64_t i = t; i < n; i += threads) {
        int r = c->mode == CPR_MODE_GYM ? run_gym_episode(c, &tab, first + i, &out[i])
                                        : run_loop_episode(c, first + i, &out[i]);
        if (r != 0) {
          rc[t] = r;
          errs[t] = g_err;
          return;
        }
      }
    } catch (std::exception& e) {
      rc[t] = -1;
      errs[t] = e.what();
    }
  };
  if (threads == 1)
    work(0);
  else {
    std::vector<std::thread> ts;
    for (int t = 0; t < threads; t++) ts.emplace_back(work, t);
    for (auto& th : ts) th.join();
  }
  for (int t = 0; t < threads; t++)
    if (rc[t] != 0) {
      g_err = errs[t];
      return rc[t];
    }
  return 0;
}

}  // extern "C"

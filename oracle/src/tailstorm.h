// TEST INFRASTRUCTURE ONLY — CPU oracle, Tailstorm part (faithful restatement).
//
//   Summary / Vote data, progress        simulator/protocols/tailstorm.ml:54-84
//   Referee (acc_votes, validity, winner, rewards)  tailstorm.ml:86-234
//   Honest node: altruistic / heuristic / optimal quorum, payload, handler
//                                        tailstorm.ml:242-609
//   n_choose_k / iter_n_choose_k         simulator/protocols/combinatorics.ml:5-32
//   SSZ'16-like attack space             simulator/protocols/tailstorm_ssz.ml:21-472
//   Gym engine                           simulator/gym/engine.ml:97-273
//
// Vertex data in the shared Block: Summary {height} = kind 0 (miner -1, work 0);
// Vote {height; depth; miner} = kind 1 with work = depth. BlockSet = Set.Make (Block)
// orders by Dag.compare_vertex (DAG depth, serial) (dag.ml:14-17).
#pragma once
#include <cstdint>
#include <functional>
#include <set>
#include <stdexcept>

#include "bk.h"
#include "des.h"

namespace oracle {

enum TsScheme { TS_CONSTANT = 0, TS_DISCOUNT = 1, TS_PUNISH = 3, TS_HYBRID = 4 };
enum TsSelection { TS_ALTRUISTIC = 0, TS_HEURISTIC = 1, TS_OPTIMAL = 2 };

// this build's policy ids (tailstorm_ssz.ml:365-472); registry order is the reverse
enum TsPolicy { TSPOL_HONEST = 0, TSPOL_GET_AHEAD = 1, TSPOL_MINOR_DELAY = 2,
                TSPOL_AVOID_LOSS = 3 /* avoid_loss_alt */, TSPOL_AVOID_LOSS_A = 4 /* avoid_loss */,
                TSPOL_AVOID_LOSS_B = 5 /* avoid_loss_alt2 */, TSPOL_LONG_DELAY = 6 };

// tailstorm_ssz.ml:22-38; event: 0 Append, 1 ProofOfWork, 2 Network
struct TsObs {
  int public_blocks, private_blocks, diff_blocks, public_votes, private_votes_inclusive,
      private_votes_exclusive, public_depth, private_depth_inclusive, private_depth_exclusive,
      event;
};
constexpr int TS_OBS_LEN = 10;

int ts_policy(int policy, const TsObs& o, int k);
// table-driven policy (include/cpr_hip.h CPR_TS_POLICY_TABLE, the B_k table layout)
constexpr int TS_POL_TABLE = 7;
constexpr int TS_POL_RANDOM = 8;  // a random Action8 per decision
struct TsTable {
  int dim = 0;
  std::vector<uint8_t> actions;
};
int ts_policy(int policy, const TsObs& o, int k, const TsTable* table);
void ts_obs_to_floats(const TsObs& o, bool unit, int k, double out[TS_OBS_LEN]);
TsObs ts_obs_of_floats(const double in[TS_OBS_LEN], bool unit, int k);

// combinatorics.ml:5-17 with OCaml's 63-bit wrap-around integer arithmetic
int64_t ocaml_n_choose_k(int64_t n, int64_t k);
// For n >= 21 the reference's n_choose_k overflows and often returns <= 100, so the
// optimal quorum brute-forces the true C(n, k) choices (e.g. 48 million for n = 38, k = 8).
// Both engines enumerate the same choices in the same order but skip prefixes that cannot
// be connected or cannot beat the best reward so far (TsView::optimal), and stop after this
// many prefixes, flagging the episode (on both sides identically)
constexpr int64_t TS_BRUTE_FORCE_BUDGET = 100000;
struct BudgetExceeded : std::runtime_error {
  BudgetExceeded() : std::runtime_error("optimal quorum: brute-force budget exceeded") {}
};
int64_t true_n_choose_k_saturated(int64_t n, int64_t k);  // saturates at INT64_MAX
// tests: the literal enumeration's budget, and a mode in which every optimal quorum is
// computed both ways and compared (compared: literal searches that completed; large: of
// those, with more than TS_BRUTE_FORCE_BUDGET choices)
extern int64_t g_ts_brute_budget;
// the pruned search's visit budget (TS_BRUTE_FORCE_BUDGET; the host fuzzer lowers it)
extern int64_t g_ts_opt_budget;
struct OptimalCheck {
  bool on = false;
  int64_t compared = 0, large = 0, mismatches = 0, unverified = 0;  // unverified: over budget
};
extern OptimalCheck g_ts_optimal_check;

struct DagCmp {
  bool operator()(const Block* a, const Block* b) const {
    if (a->depth != b->depth) return a->depth < b->depth;
    return a->serial < b->serial;
  }
};
using BlockSet = std::set<Block*, DagCmp>;
using VFilter = std::function<bool(Block*)>;

bool ts_validity(const Block* b, int k);
void ts_reward(const Block* x, int scheme, int k, std::vector<double>& r);
Block* ts_winner(const std::vector<Block*>& l);  // Referee.winner (global view)

// Honest (tailstorm.ml:242-609) and Referee pieces in node `view`'s view
struct TsView {
  const Sim* sim;
  int view;
  int k;
  int scheme;
  int selection;
  bool visible(const Block* b) const { return sim->visible(view, b); }
  bool appended_by_me(const Block* b) const {
    return b->vis[view].kind == WITHHELD || b->vis[view].kind == RELEASED;
  }
  std::vector<Block*> children(const Block* b) const;  // newest first
  std::vector<Block*> parents(const Block* b) const;
  Block* last_summary(Block* x) const;
  // acc_votes over children, expansion restricted by `vf` (puzzle_payload', next_summary')
  BlockSet votes_below(Block* b, const VFilter& vf) const;
  BlockSet confirming_votes(Block* b) const;  // unrestricted expansion
  BlockSet acc_parents(const std::vector<Block*>& l) const;  // acc_votes parents l
  double my_reward_of(const std::vector<Block*>& parents_, bool summary) const;
  bool quorum(Block* b, const VFilter& vf, std::vector<Block*>* q) const;
  bool altruistic(Block* b, const VFilter& vf, std::vector<Block*>* q) const;
  bool heuristic(Block* b, const VFilter& vf, std::vector<Block*>* q) const;
  // brute = true: the reference's literal enumeration (tests only)
  bool optimal(Block* b, const VFilter& vf, std::vector<Block*>* q, bool brute = false) const;
  Draft puzzle_payload(Block* b, const VFilter& vf) const;
  bool next_summary(Block* b, const VFilter& vf, Draft* d) const;
  int compare_blocks(const VFilter& vf, Block* a, Block* b) const;
  Block* update_head(const VFilter& vf, Block* old, Block* consider) const;
  bool summary_feasible(Block* preferred, Block* after) const;
};
int ts_compare_votes_in_block(const Block* a, const Block* b);

struct TsHonest : NodeImpl {
  Block* state = nullptr;
  int scheme = 0, selection = 1;
  TsView V() const { return TsView{sim, id, sim->bk_k, scheme, selection}; }
  Draft puzzle_payload() override;
  Action handler(Kind k, Block* b) override;
  Block* preferred() override { return state; }
};

// tailstorm_ssz.ml Agent (:162-351)
struct TsSszAgent {
  Sim* sim = nullptr;
  int my_id = 0;
  int k = 8, scheme = 1, selection = 1;
  Block* pub = nullptr;
  Block* priv = nullptr;
  std::vector<Block*> pending;
  Block* o_pub = nullptr;
  Block* o_priv = nullptr;
  Block* o_common = nullptr;
  int o_event = 1;
  TsView V() const { return TsView{sim, my_id, k, scheme, selection}; }
  void init(Block* root) {
    pub = priv = root;
    pending.clear();
  }
  Draft puzzle_payload() const;
  void prepare(Kind kd, Block* x);
  TsObs observe() const;
  Action apply(int action);
};

struct TsSszAttackerNode : NodeImpl {
  TsSszAgent agent;
  int policy = 0;
  int nrand = 0;  // TS_POL_RANDOM decisions so far
  const TsTable* table = nullptr;
  Draft puzzle_payload() override { return agent.puzzle_payload(); }
  Action handler(Kind k, Block* b) override;
  Block* preferred() override { return agent.priv; }
};

struct GymTailstorm {
  GymParams p;
  int k = 8, scheme = TS_DISCOUNT, selection = TS_HEURISTIC;
  Network net;
  int rng_mode = 0;
  OcamlRandom* ocaml = nullptr;
  uint64_t seed = 0, episode = 0;
  std::unique_ptr<SimRng> rng;
  std::unique_ptr<Sim> sim;
  TsSszAgent agent;
  long episode_steps = 0;
  double last_progress = 0, last_chain_time = 0, last_sim_time = 0, last_reward_attacker = 0,
         last_reward_defender = 0;

  GymTailstorm(const GymParams& p, int k, int scheme, int selection, int rng_mode,
               OcamlRandom* ocaml, uint64_t seed, uint64_t episode);
  void init();
  void reset(double obs[TS_OBS_LEN]);
  void observe(double obs[TS_OBS_LEN]) const;
  TsObs observe_int() const { return agent.observe(); }
  double step(int action, double obs[TS_OBS_LEN], bool* done, StepInfo* info);
  Kind skip_to_interaction(Block** blk);
};

// Simulator.loop task: node 0 = tailstorm_ssz attacker with `policy` (policy < 0: honest)
struct TsLoopResult {
  std::vector<int64_t> activations;
  std::vector<double> rewards;
  double head_time, head_progress;
  int head_height;
  int64_t n_vertices;
};
void ts_loop_task(const Network& net, int rng_mode, OcamlRandom* r, uint64_t seed,
                  uint64_t episode, int k, int scheme, int selection, int policy,
                  int activations, TsLoopResult* out, const TsTable* table = nullptr);

}  // namespace oracle

// TEST INFRASTRUCTURE ONLY — CPU oracle, B_k part (faithful restatement).
//
//   Vote / Block data, progress      simulator/protocols/bk.ml:26-48
//   Referee validity / winner / rewards  bk.ml:50-177
//   Honest node (quorum, propose)    bk.ml:185-311
//   SSZ'16-like attack space         simulator/protocols/bk_ssz.ml:21-415
//   Action8                          simulator/protocols/ssz_tools.ml:230-263
//   Gym engine                       simulator/gym/engine.ml:97-273
//
// Proof-of-work hashes are (30-bit bits, serial) pairs compared lexicographically
// (simulator.ml:123,215-221); max_pow = (max_int, max_int).
#pragma once
#include <cstdint>
#include <utility>

#include "des.h"

namespace oracle {

enum BkScheme { BK_CONSTANT = 0, BK_BLOCK = 2 };

// ssz_tools.ml:230-263 Variants.to_rank
enum BkAction {
  ADOPT_PROLONG = 0, OVERRIDE_PROLONG = 1, MATCH_PROLONG = 2, WAIT_PROLONG = 3,
  ADOPT_PROCEED = 4, OVERRIDE_PROCEED = 5, MATCH_PROCEED = 6, WAIT_PROCEED = 7
};
constexpr int BK_N_ACTIONS = 8;

// this build's policy ids (bk_ssz.ml:346-415); BKPOL_AVOID_LOSS is `avoid_loss_alt`, the
// function registered under "avoid-loss" (bk_ssz.ml:411-414)
enum BkPolicy { BKPOL_HONEST = 0, BKPOL_GET_AHEAD = 1, BKPOL_MINOR_DELAY = 2,
                BKPOL_AVOID_LOSS = 3, BKPOL_TABLE = 4, BKPOL_RANDOM = 5 };

// bk_ssz.ml:22-34, field order = record order; event: 0 Append, 1 ProofOfWork, 2 Network
struct BkObs {
  int public_blocks, private_blocks, diff_blocks, public_votes, private_votes_inclusive,
      private_votes_exclusive, lead, event;
};
constexpr int BK_OBS_LEN = 8;

// table policy over integer observations (this build's table-driven policy):
// index = (((min(pub,D-1)*D + min(priv,D-1))*(k+1) + min(pv,k))*(k+1) + min(pvi,k))*3 + event
struct BkTable {
  int dim = 0;
  int k = 0;
  std::vector<uint8_t> actions;
};
inline int64_t bk_table_size(int dim, int k) { return (int64_t)dim * dim * (k + 1) * (k + 1) * 3; }

int bk_policy(int policy, const BkObs& o, int k, const BkTable* table);
void bk_obs_to_floats(const BkObs& o, bool unit, int k, double out[BK_OBS_LEN]);
BkObs bk_obs_of_floats(const double in[BK_OBS_LEN], bool unit, int k);
void bk_obs_range(bool unit, double low[BK_OBS_LEN], double high[BK_OBS_LEN]);

using Pow = std::pair<int64_t, int64_t>;  // (bits, serial)
inline Pow bk_pow(const Block* b) { return Pow{b->pow_hash, b->serial}; }
constexpr int64_t OCAML_MAX_INT = 0x3fffffffffffffffLL;
inline Pow bk_max_pow() { return Pow{OCAML_MAX_INT, OCAML_MAX_INT}; }

// vote filters used by the reference: all (Fun.const true), Honest.appended_by_me
// (bk.ml:199-203), bk_ssz public_visibility (bk_ssz.ml:190-194)
enum VoteFilter { VF_ALL = 0, VF_MINE = 1, VF_PUBLIC = 2 };

// Honest (bk.ml:185-311) operations in node `view`'s view
struct BkView {
  const Sim* sim;
  int view;
  int k;
  bool visible(const Block* b) const { return sim->visible(view, b); }
  bool keep(const Block* b, int vf) const;
  std::vector<Block*> children(const Block* b) const;  // newest first (dag.ml:32)
  Block* last_block(Block* x) const;                    // bk.ml:78-87
  Pow leader_hash(const Block* x) const;                // bk.ml:205-215
  int confirming(const Block* b, int vf) const;         // #confirming votes passing vf
  int compare_blocks(int vf, Block* a, Block* b) const; // bk.ml:217-226
  Block* update_head(int vf, Block* old, Block* consider) const;  // bk.ml:228-231
  bool quorum(int vf, Block* b, std::vector<Block*>* q) const;    // bk.ml:233-279
  bool propose(int vf, Block* b, Draft* d) const;                 // bk.ml:288-295
  Draft puzzle_payload(Block* preferred) const;                   // bk.ml:281-286
};

struct BkHonest : NodeImpl {
  Block* state = nullptr;
  Draft puzzle_payload() override;
  Action handler(Kind k, Block* b) override;
  Block* preferred() override { return state; }
};

// Referee.winner over the global view (bk.ml:134-147)
Block* bk_winner(const std::vector<Block*>& l);

// bk_ssz.ml Agent (:148-332)
struct BkSszAgent {
  Sim* sim = nullptr;
  int my_id = 0;
  int k = 8;
  Block* pub = nullptr;
  Block* priv = nullptr;
  std::vector<Block*> pending;
  Block* o_pub = nullptr;
  Block* o_priv = nullptr;
  Block* o_common = nullptr;
  int o_event = 1;
  BkView V() const { return BkView{sim, my_id, k}; }
  void init(Block* root) {
    pub = priv = root;
    pending.clear();
  }
  Draft puzzle_payload() const { return V().puzzle_payload(priv); }
  void prepare(Kind kd, Block* x);
  BkObs observe() const;
  Action apply(int action);
};

struct BkSszAttackerNode : NodeImpl {
  BkSszAgent agent;
  int policy = 0;
  int nrand = 0;  // BKPOL_RANDOM decisions so far (Action8)
  const BkTable* table = nullptr;
  Draft puzzle_payload() override { return agent.puzzle_payload(); }
  Action handler(Kind k, Block* b) override;
  Block* preferred() override { return agent.priv; }
};

// engine.ml of_module for the bk_ssz attack space
struct GymBk {
  GymParams p;
  int k = 8;
  int scheme = BK_CONSTANT;
  Network net;
  int rng_mode = 0;
  OcamlRandom* ocaml = nullptr;
  uint64_t seed = 0, episode = 0;
  std::unique_ptr<SimRng> rng;
  std::unique_ptr<Sim> sim;
  BkSszAgent agent;
  long episode_steps = 0;
  double last_progress = 0, last_chain_time = 0, last_sim_time = 0, last_reward_attacker = 0,
         last_reward_defender = 0;

  GymBk(const GymParams& p, int k, int scheme, int rng_mode, OcamlRandom* ocaml, uint64_t seed,
        uint64_t episode);
  void init();
  void reset(double obs[BK_OBS_LEN]);
  void observe(double obs[BK_OBS_LEN]) const;
  BkObs observe_int() const { return agent.observe(); }
  double step(int action, double obs[BK_OBS_LEN], bool* done, StepInfo* info);
  Kind skip_to_interaction(Block** blk);
};

// Simulator.loop task: node 0 = bk_ssz attacker with `policy` (policy < 0: honest node 0),
// other nodes honest, on `net`; result of Simulator.head
struct BkLoopResult {
  std::vector<int64_t> activations;
  std::vector<double> rewards;
  double head_time, head_progress;
  int head_height, head_signer;
  int64_t n_vertices;
};
void bk_loop_task(const Network& net, int rng_mode, OcamlRandom* r, uint64_t seed,
                  uint64_t episode, int k, int scheme, int policy, const BkTable* table,
                  int activations, BkLoopResult* out);

}  // namespace oracle

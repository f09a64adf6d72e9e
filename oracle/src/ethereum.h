// TEST INFRASTRUCTURE ONLY — CPU oracle, Ethereum part (faithful restatement).
//
//   Byzantium parameters             simulator/protocols/ethereum.ml:19-24
//     (preference `HeaviestChain` maps to height, ethereum.ml:80-84; progress = work)
//   Referee validity / rewards       ethereum.ml:102-197
//   Honest node, uncle selection     ethereum.ml:209-297 (Compare.at_most_first heap sort)
//   SSZ-like attack space            simulator/protocols/ethereum_ssz.ml:21-538
//   Gym engine                       simulator/gym/engine.ml:97-273
#pragma once
#include <functional>

#include "des.h"

namespace oracle {

// ethereum_ssz.ml:161-277 — action index = rank(action) * 4 + own * 2 + foreign
enum EthAction { ADOPT_DISCARD = 0, ADOPT_RELEASE = 1, E_OVERRIDE = 2, E_MATCH = 3,
                 RELEASE1 = 4, E_WAIT = 5 };
constexpr int ETH_N_ACTIONS = 24;
inline int eth_action_index(int action, bool own, bool foreign) {
  return action * 4 + (own ? 2 : 0) + (foreign ? 1 : 0);
}

// policies (ethereum_ssz.ml:444-521); this build's ids
enum EthPolicy { EPOL_HONEST = 0, EPOL_SELFISH_RELEASE = 1, EPOL_SELFISH_DISCARD = 2,
                 EPOL_FN19 = 3, EPOL_FN19PKEL = 4 };

// ethereum_ssz.ml:21-45, field order = record order
struct EthObs {
  int public_height, public_work, private_height, private_work, diff_height, diff_work,
      public_orphans, private_orphans_inclusive, private_orphans_exclusive, event;
};
constexpr int ETH_OBS_LEN = 10;

int eth_policy(int policy, const EthObs& o);
// table-driven policy (include/cpr_hip.h CPR_ETH_POLICY_TABLE): action =
// table[(min(public_height, D-1) * D + min(private_height, D-1)) * 2 + event]
constexpr int ETH_POL_TABLE = 5;
constexpr int ETH_POL_RANDOM = 6;  // a random action of 24 per decision
struct EthTable {
  int dim = 0;
  std::vector<uint8_t> actions;
};
int eth_policy(int policy, const EthObs& o, const EthTable* table);
void eth_obs_to_floats(const EthObs& o, bool unit, double out[ETH_OBS_LEN]);
EthObs eth_obs_of_floats(const double in[ETH_OBS_LEN], bool unit);

// Honest.appended_by_me (ethereum.ml:221-225) in node `view`
inline bool eth_appended_by(const Block* b, int view) {
  return b->vis[view].kind == WITHHELD || b->vis[view].kind == RELEASED;
}

// Honest.puzzle_payload' (ethereum.ml:234-277) in node `view`
Draft eth_payload(const Sim& sim, int view, Block* preferred,
                  const std::function<bool(Block*)>& uncle_filter);

// Honest (ethereum.ml:209-297)
struct EthHonest : NodeImpl {
  Block* state = nullptr;
  Draft puzzle_payload() override;
  Action handler(Kind k, Block* b) override;
  Block* preferred() override { return state; }
};

// ethereum_ssz.ml Agent (:279-430)
struct EthSszAgent {
  Sim* sim = nullptr;
  int my_id = 0;
  Block* pub = nullptr;
  Block* priv = nullptr;
  bool own = true, foreign = true;  // mining rule
  std::vector<Block*> pending;
  Block* o_pub = nullptr;
  Block* o_priv = nullptr;
  Block* o_common = nullptr;
  int o_event = 0;
  void init(Block* root) {
    pub = priv = root;
    pending.clear();
    own = foreign = true;
  }
  Draft puzzle_payload() const;
  void prepare(Kind k, Block* x);
  EthObs observe() const;
  Action apply(int action);
};

struct EthSszAttackerNode : NodeImpl {
  EthSszAgent agent;
  int policy = 0;
  int nrand = 0;  // ETH_POL_RANDOM decisions so far
  const EthTable* table = nullptr;
  Draft puzzle_payload() override { return agent.puzzle_payload(); }
  Action handler(Kind k, Block* b) override;
  Block* preferred() override { return agent.priv; }
};

// engine.ml of_module for the ethereum_ssz attack space
struct GymEthereum {
  GymParams p;
  int scheme = 0;
  Network net;
  int rng_mode = 0;
  OcamlRandom* ocaml = nullptr;
  uint64_t seed = 0, episode = 0;
  std::unique_ptr<SimRng> rng;
  std::unique_ptr<Sim> sim;
  EthSszAgent agent;
  long episode_steps = 0;
  double last_progress = 0, last_chain_time = 0, last_sim_time = 0, last_reward_attacker = 0,
         last_reward_defender = 0;

  GymEthereum(const GymParams& p, int scheme, int rng_mode, OcamlRandom* ocaml, uint64_t seed,
              uint64_t episode);
  void init();
  void reset(double obs[ETH_OBS_LEN]);
  void observe(double obs[ETH_OBS_LEN]) const;
  EthObs observe_int() const { return agent.observe(); }
  double step(int action, double obs[ETH_OBS_LEN], bool* done, StepInfo* info);
  Kind skip_to_interaction(Block** blk);
};

// Simulator.loop task with an ethereum_ssz attacker (node 0) and honest nodes on `net`
struct EthLoopResult {
  int64_t activations[2];
  double rewards[2];
  double head_time, head_progress;
  int head_height, head_work;
  uint32_t diag;
};
void eth_two_agents_task(int rng_mode, OcamlRandom* r, uint64_t seed, uint64_t episode,
                         double alpha, int scheme, int policy, int activations,
                         EthLoopResult* out, const EthTable* table = nullptr);

}  // namespace oracle

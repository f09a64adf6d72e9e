/*
 * libcpr_hip — MI355X-native batched episode engine for pkel/cpr's gym hot path.
 *
 * C ABI (plain pointers and sizes, no exceptions across the boundary). Every entry
 * point returns an int status (CPR_OK = 0, negative = error); cpr_last_error() holds a
 * message for the calling thread.
 *
 * Reference interfaces each group of entry points replaces (file:line under the
 * pkel/cpr tree):
 *   cpr_version                    -> engine.cpr_lib_version   simulator/gym/cpr_gym_engine.ml:41
 *   cpr_batch_create               -> engine.create + Engine.Parameters.t + Engine.of_module
 *                                      simulator/gym/cpr_gym_engine.ml:42-89,
 *                                      simulator/gym/engine.ml:37-51,97-107
 *   cpr_reset                      -> engine.reset             cpr_gym_engine.ml:90-95, engine.ml:164-170
 *   cpr_step                       -> engine.step              cpr_gym_engine.ml:96-109, engine.ml:176-249
 *   cpr_policy_actions             -> engine.policies(...)[name](obs)
 *                                                              cpr_gym_engine.ml:110-138, engine.ml:258-261
 *   cpr_observation_spec           -> engine.n_actions / observation_low / observation_high
 *                                                              cpr_gym_engine.ml:146-162
 *   cpr_policy_name                -> keys of engine.policies  nakamoto_ssz.ml:342-350
 *   cpr_run_episodes               -> a Python loop of env.reset()/env.step(env.policy(obs))
 *                                      (experiments/rl-eval, gym/ocaml/test/test_benchmark.py:5-15)
 *                                      fused into one device launch per batch
 *   cpr_run_episodes (LOOP mode)   -> Simulator.loop ~activations + head
 *                                      simulator/lib/simulator.ml:519-543, csv_runner.ml:56-98
 *   cpr_node_outputs               -> the per-node `activations` / `reward` columns of a
 *                                      csv_runner.ml:74-79 row (Simulator state.activations,
 *                                      (Dag.data head).rewards, simulator.ml:377-388)
 *   cpr_stream_fill                -> the randomness the reference draws from OCaml Random
 *                                      (distributions.ml:17,24,90,93; simulator.ml:123),
 *                                      re-specified as a keyed Philox stream
 */
#ifndef CPR_HIP_H
#define CPR_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CPR_ABI_VERSION 11

typedef struct cpr_ctx cpr_ctx;
typedef struct cpr_batch cpr_batch;

enum cpr_status {
  CPR_OK = 0,
  CPR_E_INVALID_ARG = -1,   /* engine.ml:37-51 Failure / network.ml:63-72 Invalid_argument */
  CPR_E_UNSUPPORTED = -2,   /* configuration the device engine does not implement */
  CPR_E_HIP = -3,           /* HIP runtime error */
  CPR_E_CAPACITY = -4,      /* lane capacity exceeded */
  CPR_E_STATE = -5          /* call order violated (step before reset, ...) */
};

enum cpr_protocol {
  CPR_PROTO_NAKAMOTO = 0, /* nakamoto.ml + nakamoto_ssz.ml */
  CPR_PROTO_ETHEREUM = 1, /* ethereum.ml Byzantium + ethereum_ssz.ml (cpr_protocols.ml:39-49) */
  CPR_PROTO_BK = 2,       /* bk.ml + bk_ssz.ml (cpr_protocols.ml:53-72), k = cpr_config.k */
  CPR_PROTO_TAILSTORM = 3, /* tailstorm.ml + tailstorm_ssz.ml (cpr_protocols.ml:153-175),
                             k = cpr_config.k, selection = cpr_config.subblock_selection */
  CPR_PROTO_FC16 = 4       /* the FC'16 abstract selfish-mining model with probabilistic
                             termination, gym/rust/src/fc16.rs FC16SSZwPT: alpha, gamma,
                             horizon, policy = enum cpr_fc16_policy; fused episodes only
                             (cpr_run_episodes); max_steps caps an episode (CPR_ST_CAPACITY) */
};

/* policies of the FC16 model (fc16_lane.h); a table maps (a, h, fork) to an action name
 * CPR_FC16_WAIT .. CPR_FC16_MATCH: table[(min(a,D-1)*D + min(h,D-1))*3 + fork],
 * fork 0 irrelevant, 1 relevant, 2 active (fc16.rs:7-11) */
enum cpr_fc16_policy { CPR_FC16_POLICY_HONEST = 0, CPR_FC16_POLICY_SM1 = 1, CPR_FC16_POLICY_TABLE = 2 };
enum cpr_fc16_action { CPR_FC16_WAIT = 0, CPR_FC16_ADOPT = 1, CPR_FC16_OVERRIDE = 2, CPR_FC16_MATCH = 3 };

/* incentive schemes (ethereum.ml:3,173-197; bk.ml:3,151-176) */
enum cpr_reward_scheme {
  CPR_REWARD_CONSTANT = 0, /* Ethereum `Constant` (whitepaper): uncle 15/16;
                              B_k `Constant`: 1 per confirmed vote to its miner */
  CPR_REWARD_DISCOUNT = 1, /* Ethereum `Discount` (Byzantium): uncle (8 - dh) / 8 */
  CPR_REWARD_BLOCK = 2,    /* B_k `Block`: k to the block's signer (leader) */
  CPR_REWARD_PUNISH = 3,   /* Tailstorm `Punish`: 1 per vote on the longest vote branch */
  CPR_REWARD_HYBRID = 4    /* Tailstorm `Hybrid`: depth/k per vote on the longest branch;
                              Tailstorm also takes CONSTANT (1 per vote) and DISCOUNT (depth/k
                              per confirmed vote), tailstorm.ml:3,204-227 */
};

/* Tailstorm sub-block (quorum) selection, tailstorm.ml:4,262-507 */
enum cpr_subblock_selection {
  CPR_SELECT_ALTRUISTIC = 0,
  CPR_SELECT_HEURISTIC = 1,
  CPR_SELECT_OPTIMAL = 2 /* brute force over n-choose-k <= 100, else heuristic */
};

/* policy ids of the tailstorm_ssz attack space (tailstorm_ssz.ml:365-472) */
enum cpr_tailstorm_policy {
  CPR_TS_POLICY_HONEST = 0,
  CPR_TS_POLICY_GET_AHEAD = 1,
  CPR_TS_POLICY_MINOR_DELAY = 2,
  CPR_TS_POLICY_AVOID_LOSS = 3,   /* avoid_loss_alt, registered as "avoid-loss" */
  CPR_TS_POLICY_AVOID_LOSS_A = 4, /* avoid_loss */
  CPR_TS_POLICY_AVOID_LOSS_B = 5, /* avoid_loss_alt2 */
  CPR_TS_POLICY_LONG_DELAY = 6,
  CPR_TS_POLICY_TABLE = 7, /* Action8 = table[((((min(pub,D-1)*D + min(priv,D-1))*(k+1)
                             + min(public_votes,k))*(k+1) + min(private_votes_inclusive,k))*3
                             + event] with D = policy_table_dim (the B_k layout) */
  CPR_TS_POLICY_RANDOM = 8 /* loop tasks: a keyed random Action8 at every decision (the
                              reference's random attacker, cpr_protocols.ml:658-782) */
};

/* policy ids of the bk_ssz attack space (bk_ssz.ml:346-415; "avoid-loss" is avoid_loss_alt) */
enum cpr_bk_policy {
  CPR_BK_POLICY_HONEST = 0,
  CPR_BK_POLICY_GET_AHEAD = 1,
  CPR_BK_POLICY_MINOR_DELAY = 2,
  CPR_BK_POLICY_AVOID_LOSS = 3,
  CPR_BK_POLICY_TABLE = 4, /* action = table[((((min(pub,D-1)*D + min(priv,D-1))*(k+1)
                             + min(public_votes,k))*(k+1) + min(private_votes_inclusive,k))*3
                             + event] with D = policy_table_dim */
  CPR_BK_POLICY_RANDOM = 5 /* loop tasks: a keyed random Action8 at every decision
                              (cpr_protocols.ml:658-782) */
};

/* ssz_tools.ml:230-263 Action8, Variants.to_rank */
enum cpr_action8 {
  CPR_ADOPT_PROLONG = 0, CPR_OVERRIDE_PROLONG = 1, CPR_MATCH_PROLONG = 2, CPR_WAIT_PROLONG = 3,
  CPR_ADOPT_PROCEED = 4, CPR_OVERRIDE_PROCEED = 5, CPR_MATCH_PROCEED = 6, CPR_WAIT_PROCEED = 7
};

/* policy ids of the ethereum_ssz attack space (ethereum_ssz.ml:444-538) */
enum cpr_ethereum_policy {
  CPR_ETH_POLICY_HONEST = 0,
  CPR_ETH_POLICY_SELFISH_RELEASE = 1,
  CPR_ETH_POLICY_SELFISH_DISCARD = 2,
  CPR_ETH_POLICY_FN19 = 3,
  CPR_ETH_POLICY_FN19PKEL = 4,
  CPR_ETH_POLICY_TABLE = 5, /* action (0..23) = table[(min(public_height,D-1)*D
                              + min(private_height,D-1))*2 + event], D = policy_table_dim */
  CPR_ETH_POLICY_RANDOM = 6 /* loop tasks: a keyed random action of 24 at every decision
                               (cpr_protocols.ml:658-782) */
};

/* ethereum_ssz.ml:161-277: action = rank * 4 + own * 2 + foreign, rank in
 * {Adopt_discard, Adopt_release, Override, Match, Release1, Wait} */
enum cpr_ethereum_action_rank {
  CPR_ETH_ADOPT_DISCARD = 0, CPR_ETH_ADOPT_RELEASE = 1, CPR_ETH_OVERRIDE = 2,
  CPR_ETH_MATCH = 3, CPR_ETH_RELEASE1 = 4, CPR_ETH_WAIT = 5
};

enum cpr_network {
  CPR_NET_SELFISH_MINING = 0, /* network.ml:61-105, as the gym builds it (engine.ml:100-107) */
  CPR_NET_TWO_AGENTS = 1,     /* network.ml:50-59 */
  CPR_NET_HONEST_CLIQUE = 2,  /* experiments/simulate/models.ml:3-28 honest_clique: `defenders`
                                 = n honest nodes (2..64), node i has compute i + 1, every
                                 link delay uniform [delay_lo, delay_hi), simple
                                 dissemination; CPR_MODE_LOOP, Nakamoto or Ethereum */
  CPR_NET_EXP_CLIQUE = 3,     /* Network.T.symmetric_clique with exponential propagation
                                 (cpr_protocols.ml:200-210,478-485): node 0 (the attacker,
                                 running cfg.policy) plus `defenders` honest nodes (1..63),
                                 equal compute, every link delay exponential with mean
                                 propagation_delay; CPR_MODE_LOOP, every protocol
                                 (Nakamoto on the exact event engine in Nakamoto mode) */
  CPR_NET_ABSTRACT_GAMMA = 4  /* FLAGGED abstract-gamma mode (not a network
                                 of the reference, which rejects gamma = 1, envs.py:73-75):
                                 the gym's attacker + `defenders` equal-compute honest nodes
                                 with zero propagation delays, where a release that ties the
                                 window's fresh defender block wins at each defender, its
                                 miner included, iff that defender's coin
                                 U(k, 0, j) < gamma (Eyal-Sirer'14 gamma, exact for any
                                 gamma in [0, 1]); every other tie keeps the first-received
                                 block. Nakamoto, CPR_MODE_GYM; no replay, no node outputs */
};

enum cpr_mode {
  CPR_MODE_GYM = 0,  /* episode = reset + steps until done (engine.ml:209-214) */
  CPR_MODE_LOOP = 1  /* episode = Simulator.loop ~activations (simulator.ml:519-533) */
};

/* policy ids of the nakamoto_ssz attack space, nakamoto_ssz.ml:274-350 */
enum cpr_policy {
  CPR_POLICY_HONEST = 0,
  CPR_POLICY_SIMPLE = 1,
  CPR_POLICY_EYAL_SIRER_2014 = 2,
  CPR_POLICY_SAPIRSHTEIN_2016_SM1 = 3,
  CPR_POLICY_TABLE = 4, /* action = table[(min(pub,D-1)*D + min(priv,D-1))*2 + event] */
  CPR_POLICY_RANDOM = 5 /* loop tasks on the event engine (cpr_protocols.ml:658-782): a keyed
                           random action of 4 at every decision; the i-th decision of an
                           episode draws word 0 of Philox block (i, 0x50000000) and takes
                           (w0 * n) >> 32 (every protocol's *_POLICY_RANDOM likewise) */
};

/* nakamoto_ssz.ml:116-154, Variants.to_rank */
enum cpr_nakamoto_action { CPR_ADOPT = 0, CPR_OVERRIDE = 1, CPR_MATCH = 2, CPR_WAIT = 3 };

/* per-episode status bits */
enum cpr_episode_status {
  CPR_ST_OK = 0u,
  CPR_ST_TIE = 1u,      /* a defender resolved an equal-time, equal-height delivery */
  CPR_ST_OVERLAP = 2u,  /* Nakamoto: an activation fired while finite-delay messages were in
                           flight; the episode is re-run exactly (CPR_ST_EXACT_RERUN) */
  CPR_ST_DEEP_FORK = 4u,      /* Nakamoto: private chain beyond its slots */
  CPR_ST_TIE_UNRESOLVED = 8u, /* Nakamoto: tie replay capacity exceeded */
  CPR_ST_STALE_TIME = 16u,    /* Nakamoto: head time older than the time log */
  CPR_ST_CAPACITY = 32u,      /* event-engine lanes (Ethereum, B_k, Tailstorm): a lane
                                 capacity (vertex ring, event heap, candidate lists, frontier,
                                 Tailstorm brute-force budget) was exceeded; the episode's
                                 outputs are not valid */
  CPR_ST_REFERENCE_RAISES = 64u, /* Tailstorm: the reference raises an exception at this point
                                 (List.for_all2 in summary dedup, Division_by_zero in
                                 n_choose_k, assert false in heuristic_quorum); the episode
                                 stops, outputs not valid */
  CPR_ST_TRACE_MISS = 128u,     /* cpr_replay: the episode needed a draw its trace does not
                                 hold (too few activations, a missing delay key); outputs
                                 not valid */
  CPR_ST_EXACT_RERUN = 256u     /* Nakamoto fused episodes (cpr_run_episodes, cpr_replay) and
                                 lockstep lanes (cpr_step): the closed-form lane flagged the
                                 episode (OVERLAP, DEEP_FORK, TIE_UNRESOLVED, STALE_TIME) and it
                                 was simulated again on the exact event engine (DESIGN.md
                                 §4.3); its outputs are that re-run's, and the lane's flags
                                 are kept beside this bit */
};

/* status bits that make an episode's outputs invalid; such episodes never enter a
 * summary's sums (cpr_summary.invalid counts them). A Nakamoto lockstep lane (cpr_step)
 * whose step sets OVERLAP, DEEP_FORK, TIE_UNRESOLVED or STALE_TIME is simulated again on the
 * exact event engine from its first draw and the actions it was given, and stays there
 * until its next reset: its outputs are exact and its status carries CPR_ST_EXACT_RERUN
 * beside those bits. Only a lane that cannot move (all exact slots of the batch in use, an
 * episode longer than its action log, a network the exact engine does not hold) reports
 * the bits without CPR_ST_EXACT_RERUN, and its outputs are then not exact. */
#define CPR_ST_INVALID (CPR_ST_CAPACITY | CPR_ST_REFERENCE_RAISES | CPR_ST_TRACE_MISS)
#define CPR_ST_LOCKSTEP_INEXACT \
  (CPR_ST_OVERLAP | CPR_ST_DEEP_FORK | CPR_ST_TIE_UNRESOLVED | CPR_ST_STALE_TIME)

typedef struct cpr_config {
  int32_t protocol;          /* enum cpr_protocol */
  int32_t network;           /* enum cpr_network */
  int32_t mode;              /* enum cpr_mode */
  int32_t policy;            /* enum cpr_policy; for cpr_step lanes the caller acts */
  const uint8_t* policy_table; /* host pointer: the *_POLICY_TABLE of the protocol */
  int32_t policy_table_dim;
  int32_t unit_observation;  /* ssz_tools.ml NormalizeObs ~unit */
  double alpha;              /* attacker compute, [0,1] */
  double gamma;              /* selfish-mining gamma, [0,1] */
  int32_t defenders;         /* >= 2 for CPR_NET_SELFISH_MINING */
  int32_t reward_scheme;     /* enum cpr_reward_scheme (Ethereum) */
  double activation_delay;   /* expected block interval, > 0 */
  double propagation_delay;  /* defender<->defender delay; the gym uses 1e-9 */
  int64_t max_steps;         /* GYM mode termination; <= 0 means max_int */
  double max_progress;       /* GYM mode termination; <= 0 means +inf */
  double max_time;           /* GYM mode termination; <= 0 means +inf */
  int64_t activations;       /* LOOP mode: activations per episode */
  uint64_t seed;             /* keyed-stream seed */
  int64_t n_lanes;           /* lockstep lanes for cpr_reset/cpr_step; 0 = none */
  int32_t k;                 /* B_k / Tailstorm: votes per block (bk.ml:7), >= 1 */
  int32_t subblock_selection;/* Tailstorm: enum cpr_subblock_selection */
  double delay_lo, delay_hi;  /* CPR_NET_HONEST_CLIQUE link delays U[lo, hi); NaN, NaN = the
                                 models.ml default 0.5, 1.5 (0, 0 is a real zero delay) */
  double horizon;             /* CPR_PROTO_FC16: expected progress before termination, >= 1 */
} cpr_config;

/* one finished episode; identical layout is produced by the CPU oracle */
typedef struct cpr_episode_record {
  double reward_attacker;    /* head.rewards[0]              engine.ml:215-219 */
  double reward_defender;    /* sum of head.rewards[1..]     */
  double progress;           /* Ref.progress head            engine.ml:208 */
  double chain_time;         /* Simulator.timestamp head     simulator.ml:14-21 */
  double sim_time;           /* clock.now                    */
  int64_t n_steps;           /* episode_n_steps              engine.ml:236 */
  int64_t n_activations;     /* episode_n_activations        engine.ml:237 */
  int32_t head_height;
  int32_t head_miner;        /* -1 = n/a (genesis); B_k: the head block's signer (leader) */
  uint32_t status;           /* enum cpr_episode_status bits */
  int32_t head_work;         /* Ethereum head work (ethereum.ml:93-97); 0 for Nakamoto */
} cpr_episode_record;

#define CPR_HIST_BINS 64

/* batch reduction; integer-exact so 1/2/4/8-GPU totals are bit-identical */
typedef struct cpr_summary {
  int64_t episodes;
  int64_t steps;
  int64_t activations;
  int64_t reward_attacker_fx;   /* sum of reward_attacker * 2^20 */
  int64_t reward_defender_fx;   /* sum of reward_defender * 2^20 */
  int64_t progress_fx;          /* sum of progress * 2^20 */
  uint64_t rel_revenue_fx;      /* sum of round(attacker/(attacker+defender) * 2^32) */
  uint64_t rel_revenue_sq_fx;   /* sum of round((attacker/(attacker+defender))^2 * 2^32) */
  int64_t orphans;              /* activations - head height */
  /* status_tie / status_overlap are diagnostics of the route that ran: the closed-form
     Nakamoto lane and the Ethereum window lane set CPR_ST_TIE when they replay a
     same-instant race and CPR_ST_OVERLAP when they hand an episode to the exact re-run;
     the per-lane event engines follow the reference's queue and set neither. Every other
     field is route-independent. */
  int64_t status_tie;           /* episodes with CPR_ST_TIE */
  int64_t status_overlap;       /* episodes with CPR_ST_OVERLAP */
  int64_t status_other;         /* valid episodes with other status bits */
  int64_t hist[CPR_HIST_BINS];  /* relative revenue histogram, bin = floor(rel*64) */
  int64_t invalid;              /* episodes with CPR_ST_INVALID bits: counted here and in
                                   steps / activations only, never in episodes or any sum */
} cpr_summary;

/* lockstep info, structure of arrays, one entry per lane (engine.ml:224-241) */
typedef struct cpr_step_info {
  double* episode_reward_attacker;
  double* episode_reward_defender;
  double* episode_progress;
  double* episode_chain_time;
  double* episode_sim_time;
  int64_t* episode_n_steps;
  int64_t* episode_n_activations;
  int32_t* head_height;
  int32_t* head_miner;
  uint32_t* status;  /* cpr_episode_status bits of the lane's episode (CPR_ST_INVALID: the
                        reference would have raised / the lane's capacity was exceeded;
                        CPR_ST_LOCKSTEP_INEXACT without CPR_ST_EXACT_RERUN: Nakamoto
                        outputs not exact) */
} cpr_step_info;

/* An exported activation/delay trace: every random draw of n_episodes
 * episodes, addressed by the coordinates of the keyed stream, so an episode replays
 * bit-exactly on any engine that consumes the same draws. Arrays are CSR over episodes
 * (x_offset has n_episodes + 1 entries, x_offset[0] = 0); all host pointers.
 *   act_miner[j], act_delay[j]  activation j's miner (the alias sample over compute shares,
 *                               distributions.ml:45-98 via simulator.ml:465-472) and the
 *                               exponential delay drawn when clock j is scheduled
 *                               (simulator.ml:170-173; j = 0 is the first clock)
 *   pow_hash[s]                 30-bit Random.bits of vertex serial s (simulator.ml:123);
 *                               B_k and Tailstorm only (may be empty otherwise)
 *   link_key[i], link_delay[i]  message delays drawn at Network Tx (simulator.ml:481-487),
 *                               keys ascending per episode:
 *                               Nakamoto, Ethereum: (kw << 32) | (off << 12) | dest with
 *                                 kw = activations when the share happened, off = the
 *                                 message's position in that share's order
 *                               B_k, Tailstorm: (serial << 32) | dest
 * Traces come from the CPU oracle (tests/oracle_py.py export_traces; with the OCaml 4.12
 * Random replica it records the reference's own stream) or from an instrumented OCaml
 * Simulator. */
typedef struct cpr_trace {
  int64_t n_episodes;
  const int64_t* act_offset;
  const int32_t* act_miner;
  const double* act_delay;
  const int64_t* pow_offset;
  const int32_t* pow_hash;
  const int64_t* link_offset;
  const uint64_t* link_key;
  const double* link_delay;
} cpr_trace;

const char* cpr_version(void);
int cpr_abi_version(void);
const char* cpr_last_error(void);

/* device_ordinal: HIP device index (one context per GPU / per process) */
int cpr_ctx_create(int device_ordinal, cpr_ctx** out);
int cpr_ctx_destroy(cpr_ctx* ctx);
int cpr_device_count(int* out);

int cpr_batch_create(cpr_ctx* ctx, const cpr_config* cfg, cpr_batch** out);
int cpr_batch_destroy(cpr_batch* b);

/* Run episodes [first_episode, first_episode + n_episodes) to completion on the device.
 * summary: host pointer, accumulated (+=) — zero it before the first call.
 * records: NULL, or n_episodes records; records_on_device != 0 means a device pointer.
 * Synchronous. */
int cpr_run_episodes(cpr_batch* b, int64_t n_episodes, uint64_t first_episode,
                     cpr_summary* summary, cpr_episode_record* records,
                     int records_on_device);
/* Same, asynchronous on the context's streams; summary must be a device pointer to a
 * zeroed cpr_summary and records (optional) a device pointer. Both are complete after
 * cpr_synchronize (Nakamoto: exact re-runs of flagged episodes, CPR_ST_EXACT_RERUN, run on
 * the context's stream at the next flush). Blocking point: a flush (cpr_synchronize, or one
 * forced inside this call when the context's re-run table or overflow-flag chunks are full)
 * waits for the stream to read how many episodes were queued, so that it can size the
 * re-run grid; an _async call that forces one therefore returns only after the launches
 * before it have finished. */
int cpr_run_episodes_async(cpr_batch* b, int64_t n_episodes, uint64_t first_episode,
                           cpr_summary* summary_dev, cpr_episode_record* records_dev);
int cpr_synchronize(cpr_ctx* ctx);
/* Replay trace episodes [0, trace->n_episodes) on the device with the batch's protocol,
 * mode and policy (fused episodes, like cpr_run_episodes, drawing from the trace instead
 * of the keyed stream); records[e] is trace episode e. summary (host) is accumulated (+=).
 * records: NULL or n_episodes records (device pointer if records_on_device != 0).
 * Replaces nothing in the reference directly: it is the cross-engine check the north star
 * asks for (same exported trace -> same per-episode outcomes). Synchronous. */
int cpr_replay(cpr_batch* b, const cpr_trace* trace, cpr_summary* summary,
               cpr_episode_record* records, int records_on_device);
/* Per-node outputs of episodes: activations per node and the head's reward array, one row
 * of n_nodes per episode (node 0 = the attacker on selfish-mining / two-agents networks;
 * n_nodes must be the network's node count: 2, defenders + 1, or defenders for cliques).
 * trace == NULL: keyed-stream episodes [first_episode, first_episode + n_episodes); else
 * trace episodes [0, trace->n_episodes) (n_episodes / first_episode ignored). The episodes
 * run on the exact event engine (Nakamoto configurations of the closed-form lane: the
 * Nakamoto-mode engine of its exact re-runs), so results equal cpr_run_episodes /
 * cpr_replay bit for bit. Host buffers: node_activations and node_rewards
 * [n_episodes][n_nodes]; records (optional) [n_episodes] as cpr_run_episodes, except that
 * head_miner is the head block's miner in LOOP mode too (nakamoto.ml:22-27 head info;
 * -1 genesis, Tailstorm summaries). Not for FC16. Synchronous. */
int cpr_node_outputs(cpr_batch* b, int64_t n_episodes, uint64_t first_episode,
                     const cpr_trace* trace, int32_t n_nodes, cpr_episode_record* records,
                     int64_t* node_activations, double* node_rewards);
/* device time (HIP events on the context's stream) of the last episode-kernel launch of
 * this batch, and the activations it simulated (valid after cpr_run_episodes returns;
 * after cpr_run_episodes_async + cpr_synchronize the time is valid and activations is -1) */
int cpr_last_launch(cpr_batch* b, double* kernel_ms, int64_t* activations);
/* shape of the last episode-kernel launch of this batch (fused episodes, replay, rollout):
 * lanes = device lanes launched; resident = lanes the device holds at once for that kernel
 * (occupancy API x CUs x 256, before the HBM budget and the episode count cap the launch).
 * Before any launch lanes = 0 and resident is the fused-episode kernel's figure.
 * Diagnostic for bench.py (lanes / resident), no reference counterpart. ABI v9. */
int cpr_launch_shape(cpr_batch* b, int64_t* lanes, int64_t* resident);
/* cumulative count of exact Nakamoto re-runs on this context whose episode outgrew the
 * LDS-resident event heap and ran again with the heap in HBM (k_nak_exact_rerun's second
 * attempt). Synchronizes the context's stream. Diagnostic, no reference counterpart. ABI v9. */
int cpr_rerun_hbm_retries(cpr_ctx* ctx, int64_t* retries);
/* cumulative exact re-runs on this context: episodes the fused kernels flagged (closed-form
 * Nakamoto overlaps, deep forks and unresolved ties; Ethereum window-lane hand-backs) and
 * re-ran on the exact event engine, the flushes that ran them and those flushes' kernel
 * milliseconds (HIP events on the context's stream). Synchronizes the stream if a flush is
 * pending. Diagnostic for bench.py, no reference counterpart. Since ABI v10. */
int cpr_rerun_stats(cpr_ctx* ctx, int64_t* episodes, int64_t* flushes, double* ms);
/* exact-replay coverage of this batch's lockstep lanes (Nakamoto closed-form lanes that
 * leave the closed form continue on the exact engine from an action log): log_steps = the
 * steps of each lane's action log, exact_slots = the engine slots shared by the lanes (both
 * 0 before the first cpr_reset, or where no lane can leave the closed form). A lane whose
 * episode is past log_steps, or that finds every slot taken, when it leaves the closed form
 * keeps the closed form's status flags (not exact); log_steps < max_steps happens only
 * beyond 4 GiB of logs (lanes x episode length). Diagnostic, no reference counterpart.
 * ABI v11. */
int cpr_lockstep_coverage(cpr_batch* b, int64_t* log_steps, int64_t* exact_slots);

/* Lockstep env API over cfg->n_lanes lanes (host pointers).
 * reset: lanes with mask[i] != 0 (mask NULL = all) start episode episode_ids[i]
 *        (episode_ids NULL = lane index); obs gets obs_len doubles per lane.
 * step:  actions[i] in [0, n_actions); writes obs, reward (engine.ml:223), done, info. */
int cpr_reset(cpr_batch* b, const uint8_t* mask, const uint64_t* episode_ids, double* obs);
int cpr_step(cpr_batch* b, const int32_t* actions, double* obs, double* reward,
             uint8_t* done, cpr_step_info* info);
/* integer observation fields of every lane: Nakamoto (public, private, diff, event);
 * B_k the 8 bk_ssz fields (bk_ssz.ml:22-34) */
int cpr_observe_fields(cpr_batch* b, int32_t* fields);

/* Lockstep rollout on the device (B_k): every one of cfg->n_lanes lanes takes n_steps
 * steps with the batch policy (cfg->policy, built-in or table) evaluated on the device;
 * a lane whose episode ends restarts at episode id (previous id + n_lanes), like a gym
 * VecEnv auto-reset (the observation written at a done step is the new episode's first).
 * Continues from the lanes' current state (a first call without cpr_reset starts lane i at
 * episode i). Outputs are optional, step-major:
 *   obs [n_steps][n_lanes][obs_len] f64, reward [n_steps][n_lanes] f64 (engine.ml:223),
 *   done [n_steps][n_lanes] u8; device pointers if outputs_on_device != 0, else host
 *   pointers (staged through library-owned device buffers).
 * summary (host, accumulated): steps / activations of the whole rollout, the other fields
 * over the episodes that finished in it. Synchronous; cpr_last_launch times the kernel.
 * Replaces SB3 SubprocVecEnv rollouts over cpr_gym envs (experiments/train/ppo.py:278-285). */
int cpr_rollout(cpr_batch* b, int64_t n_steps, double* obs, double* reward, uint8_t* done,
                int outputs_on_device, cpr_summary* summary);

/* policy evaluated on encoded observations (host): obs n x obs_len -> actions n */
int cpr_policy_actions(cpr_batch* b, int32_t policy, const double* obs, int64_t n,
                       int32_t* actions);

int cpr_observation_spec(cpr_batch* b, int32_t* obs_len, int32_t* n_actions, double* low,
                         double* high);
/* policy names in the reference's registry order (Collection prepends): index -> name */
int cpr_policy_count(int32_t protocol);
const char* cpr_policy_name(int32_t protocol, int32_t index, int32_t* policy_id);

/* Keyed stream: out[4*i..4*i+3] = Philox4x32-10 block of
 * ctr = (episode_lo, episode_hi, idx0 + i, tag), key = (seed_lo, seed_hi), computed on
 * the device; exp_out (optional) = -log(u53(w2,w3)) of each block via cpr_log. */
int cpr_stream_fill(cpr_ctx* ctx, uint64_t seed, uint64_t episode, uint32_t idx0,
                    uint32_t tag, int64_t n, uint32_t* out, double* exp_out);

#ifdef __cplusplus
}
#endif

#endif /* CPR_HIP_H */

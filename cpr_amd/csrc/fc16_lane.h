// One GPU lane = one episode of the FC'16 abstract selfish-mining model with probabilistic
// termination, gym/rust/src/fc16.rs FC16SSZwPT: the Sapirshtein et
// al. Bitcoin MDP as an environment, the model the reference's MDP toolbox solves
// (mdp/lib/models/fc16sapirshtein.py) and cpr_amd.mdp restates. State (a, h, fork); the
// actions offered in a state are the list [Wait, Adopt, Override if a > h, Match if
// a >= h] (fc16.rs:50-60); an episode ends when a Bernoulli(1/horizon) draw per unit of
// progress fires (fc16.rs:178-190, Bar-Zur et al. AFT'20).
//
// Randomness from the keyed stream, tag TAG_FC16:
//   start            block(0, TAG_FC16 | 1).w0 < t_alpha -> (1, 0) else (0, 1)
//   step j           block(j, TAG_FC16): w0 < t_alpha mining (attacker finds the block),
//                    w1 < t_gamma network (the defender block loses the match race)
//   termination i    word i & 3 of block(j, TAG_FC16 | 0x100000 | i >> 2) < t_term
// Thresholds are floor(p * 2^32), so each draw is an exact integer compare on both the
// device and the oracle (tests/oracle_py.py fc16_episode).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "cpr_stream.h"

namespace cpr {
namespace fc16 {

constexpr uint32_t TAG_FC16 = 0x40000000u;
enum : int32_t { IRRELEVANT = 0, RELEVANT = 1, ACTIVE = 2 };
// action names (fc16.rs:19-25); a policy returns a name, the lane maps it to the offered list
enum : int32_t { WAIT = 0, ADOPT = 1, OVERRIDE = 2, MATCH = 3 };
enum : int32_t { POLICY_HONEST = 0, POLICY_SM1 = 1, POLICY_TABLE = 2 };

struct Fc16Params {
  uint64_t t_alpha, t_gamma, t_term;  // floor(p * 2^32)
  int64_t max_steps;                  // truncation cap (the reference env never truncates)
  int32_t policy, table_dim;
  const uint8_t* table;               // [(min(a,D-1) * D + min(h,D-1)) * 3 + fork] -> name
};

struct Fc16Out {
  int64_t reward, progress, steps;
  int32_t a, h, fork;
  uint32_t status;  // CPR_ST_CAPACITY (32) if truncated at max_steps
};

__host__ __device__ inline int32_t fc16_policy(const Fc16Params& P, int32_t a, int32_t h,
                                               int32_t fork) {
  switch (P.policy) {
    case POLICY_HONEST:  // mine on the longest chain, publish at once
      return a > h ? OVERRIDE : (h > a ? ADOPT : WAIT);
    case POLICY_SM1:  // sapirshtein-2016-sm1 (nakamoto_ssz.ml:325-339) on (h, a)
      if (h > a) return ADOPT;
      if (h == 1 && a == 1) return MATCH;
      if (h == a - 1 && h >= 1) return OVERRIDE;
      return WAIT;
    default: {
      const int32_t D = P.table_dim;
      const int32_t ac = a >= D ? D - 1 : a, hc = h >= D ? D - 1 : h;
      return (int32_t)P.table[(ac * D + hc) * 3 + fork];
    }
  }
}

template <class St>
__host__ __device__ inline Fc16Out fc16_episode(const Fc16Params& P, const St& S) {
  Fc16Out o{0, 0, 0, 0, 0, IRRELEVANT, 0u};
  if ((uint64_t)S.block(0, TAG_FC16 | 1u).w0 < P.t_alpha)
    o.a = 1;
  else
    o.h = 1;
  for (uint32_t j = 0;; ++j) {
    if ((int64_t)j >= P.max_steps) {
      o.status |= 32u;
      return o;
    }
    // the named action if the state offers it, else the list's first entry Wait
    // (fc16.rs:182: an out-of-range index acts as index 0)
    int32_t act = fc16_policy(P, o.a, o.h, o.fork);
    if ((act == OVERRIDE && !(o.a > o.h)) || (act == MATCH && !(o.a >= o.h))) act = WAIT;
    const Words4 w = S.block(j, TAG_FC16);
    const bool mining = (uint64_t)w.w0 < P.t_alpha;
    int32_t na, nh, nf, r = 0, g = 0;
    if (act == ADOPT) {  // fc16.rs:131-137
      na = mining ? 1 : 0;
      nh = mining ? 0 : 1;
      nf = IRRELEVANT;
      g = o.h;
    } else if (act == OVERRIDE) {  // fc16.rs:116-129
      na = mining ? o.a - o.h : o.a - o.h - 1;
      nh = mining ? 0 : 1;
      nf = mining ? IRRELEVANT : RELEVANT;
      r = g = o.h + 1;
    } else if (act == MATCH || o.fork == ACTIVE) {  // fc16.rs:103-114
      if (mining) {
        na = o.a + 1;
        nh = o.h;
        nf = ACTIVE;
      } else if ((uint64_t)w.w1 < P.t_gamma) {
        na = o.a - o.h;
        nh = 1;
        nf = RELEVANT;
        r = o.h;
      } else {
        na = o.a;
        nh = o.h + 1;
        nf = RELEVANT;
      }
    } else {  // Wait, no active match, fc16.rs:94-101
      na = mining ? o.a + 1 : o.a;
      nh = mining ? o.h : o.h + 1;
      nf = mining ? IRRELEVANT : RELEVANT;
    }
    o.a = na;
    o.h = nh;
    o.fork = nf;
    o.reward += r;
    o.progress += g;
    o.steps += 1;
    // probabilistic termination: one Bernoulli(1/horizon) per unit of progress
    bool term = false;
    for (int32_t i = 0; i < g && !term; i += 4) {
      const Words4 t = S.block(j, TAG_FC16 | 0x100000u | (uint32_t)(i >> 2));
      const uint32_t tw[4] = {t.w0, t.w1, t.w2, t.w3};
      for (int32_t q = 0; q < 4 && i + q < g; ++q) term |= (uint64_t)tw[q] < P.t_term;
    }
    if (term) return o;
  }
}

}  // namespace fc16
}  // namespace cpr

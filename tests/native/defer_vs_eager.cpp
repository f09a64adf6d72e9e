// TEST INFRASTRUCTURE ONLY. The d = 2 summary-only kernel's deferred races
// (NakLane::resolve<.., TT = 2> + verify_races, cpr_amd/csrc/nakamoto_lane.h) against the
// eager closed form (resolve<.., TT = 1>) on the host: the same episodes, with the gym loop
// of k_run_episodes (kernels.hip run_gym, as a wave of one lane: the race list is the
// lane's own, verified when full; list sizes 6 and 64), must end in the same lane state
// word for word (NakLane::pack) and the same head, unless the verification flagged the
// episode for the eager second pass (ST_RACE_REDO; the kernel then discards the deferred
// run), which it must do exactly when a race went otherwise than assumed.
// Configurations with dmax > delta make races go the other way often, so the flagging is
// exercised; a tiny delta makes same-instant ties common.
// Prints one JSON summary line; exit code 1 on any difference.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../cpr_amd/csrc/nakamoto_lane.h"
#include "../../oracle/src/keyed_stream.h"

using namespace cpr;

struct Cfg {
  double alpha, delta, dmax;
  int policy;  // 0..3 (nak_policy)
  int steps;
};

struct Run {
  std::vector<uint32_t> words;
  BRef head;
  long drains = 0, rollbacks = 0, races = 0;
};

struct Deferred {
  std::vector<uint4> rq;
  int32_t flag = 0;
  uint32_t ep[2] = {0u, 0u};
  Deferred(const Deferred&) = delete;
  LaneMem M;
  Deferred(const NakParams& P, int32_t cap) : rq(cap) {
    M.times = false;
    M.cap = P.cap;
    M.rq = rq.data();
    M.rq_cap = cap;
    M.rflag = &flag;
    M.rep = ep;
    M.lane = 0;
  }
};

template <int POL, int TT>
static Run run(const NakParams& P, const Stream& S, int32_t cap) {
  Deferred D(P, cap);
  const LaneMem& M = D.M;
  Run r;
  NakLane L;
  L.init();
  L.activate(P, S, M);
  for (int64_t s = 0; s < P.max_steps; ++s) {
    const NakLane::Draw dr = L.draw(P, S);
    L.apply(L.policy_action<POL>(P));
    const int32_t q0 = L.qn;
    L.resolve<Stream, 0, TT>(P, S, M);
    if (TT == 2) enqueue_race(L, M);
    r.races += L.qn - q0;
    L.activate(P, S, M, dr);
    if (TT == 2 && races_due(L, M)) {
      verify_races(L, P, S, M);
      ++r.drains;
    }
  }
  if (TT == 2) verify_races(L, P, S, M);
  std::vector<uint32_t> w(CK_WORDS);
  L.pack(w.data());
  r.words = w;
  r.head = L.head(P, M);
  return r;
}

// verifications counted by outcome: a redo flag (a race the release did not win, or a tie
// the closed-form rule decides otherwise) or a tie kept as assumed
template <int POL>
static void count_outcomes(const NakParams& P, const Stream& S, int32_t cap, long* rollbacks,
                           long* kept) {
  Deferred D(P, cap);
  const LaneMem& M = D.M;
  NakLane L;
  L.init();
  L.activate(P, S, M);
  auto verify = [&]() {
    races_publish(S, M);
    races_check(L, P, S, M);
    *rollbacks += (D.flag & 2) ? 1 : 0;
    *kept += D.flag == 1 ? 1 : 0;
    races_settle(L, M);
  };
  for (int64_t s = 0; s < P.max_steps; ++s) {
    const NakLane::Draw dr = L.draw(P, S);
    L.apply(L.policy_action<POL>(P));
    L.resolve<Stream, 0, 2>(P, S, M);
    enqueue_race(L, M);
    L.activate(P, S, M, dr);
    if (races_due(L, M)) verify();
  }
  verify();
}

// a wave of W lanes emulated phase by phase (kernels.hip run_gym + enqueue_race +
// verify_races with the list shared by the lanes): lane i runs episode ep0 + i; every lane
// must end as its eager run does. Returns the lanes that differ.
template <int POL>
static int run_wave(const NakParams& P, uint64_t ep0, int W, int32_t per_lane, long* drains) {
  const uint64_t seed = 0x5eed0000ull;
  std::vector<uint4> rq(W * per_lane);
  std::vector<int32_t> flag(W, 0);
  std::vector<uint32_t> rep(2 * W);
  std::vector<LaneMem> M(W);
  std::vector<Stream> S(W);
  std::vector<NakLane> L(W);
  for (int i = 0; i < W; ++i) {
    const uint64_t ep = ep0 + i;
    S[i] = Stream{(uint32_t)seed, (uint32_t)(seed >> 32), (uint32_t)ep, (uint32_t)(ep >> 32)};
    M[i].times = false;
    M[i].cap = P.cap;
    M[i].rq = rq.data();
    M[i].rq_cap = W * per_lane;
    M[i].rflag = flag.data();
    M[i].rep = rep.data();
    M[i].lane = i;
    M[i].wave = W;
    L[i].init();
    L[i].activate(P, S[i], M[i]);
  }
  auto drain = [&]() {
    for (int i = 0; i < W; ++i) races_publish(S[i], M[i]);
    for (int i = 0; i < W; ++i) races_check(L[i], P, S[i], M[i]);
    for (int i = 0; i < W; ++i) races_settle(L[i], M[i]);
    ++*drains;
  };
  std::vector<NakLane::Draw> dr(W);
  for (int64_t s = 0; s < P.max_steps; ++s) {
    for (int i = 0; i < W; ++i) {
      dr[i] = L[i].draw(P, S[i]);
      L[i].apply(L[i].policy_action<POL>(P));
      L[i].resolve<Stream, 0, 2>(P, S[i], M[i]);
    }
    int32_t below = 0;  // enqueue_race: the racing lanes in lane order after the list
    for (int i = 0; i < W; ++i)
      if (L[i].rw) rq[L[i].qn + below++] = race_entry(L[i], i);
    for (int i = 0; i < W; ++i) {
      L[i].qn += below;
      L[i].rw = 0u;
      L[i].activate(P, S[i], M[i], dr[i]);
    }
    if (races_due(L[0], M[0])) drain();
  }
  drain();
  int bad = 0;
  for (int i = 0; i < W; ++i) {
    if (L[i].status & ST_RACE_REDO) continue;  // the eager second pass runs it
    const Run a = run<POL, 1>(P, S[i], per_lane);
    std::vector<uint32_t> w(CK_WORDS);
    L[i].pack(w.data());
    bad += w != a.words ? 1 : 0;
  }
  return bad;
}

template <int POL>
static bool compare(const Cfg& cf, uint64_t ep, long* races, long* drains, long* rollbacks,
                    long* kept, long* ties, long* unresolved, long* redo) {
  NakParams P{};
  P.t_att = oracle::alpha_threshold(cf.alpha);
  P.d = 2;
  P.ev = 1.0;
  P.delta = cf.delta;
  P.dmax = cf.dmax;
  P.arrive = 1;
  P.max_steps = cf.steps;
  P.max_progress = __builtin_inf();
  P.max_time = __builtin_inf();
  P.policy = POL;
  P.cap = cf.steps + 64;
  const uint64_t seed = 0x5eed0000ull;
  const Stream S{(uint32_t)seed, (uint32_t)(seed >> 32), (uint32_t)ep, (uint32_t)(ep >> 32)};
  const int32_t cap = (ep & 1) ? 64 : 6;
  const Run a = run<POL, 1>(P, S, cap);
  const Run b = run<POL, 2>(P, S, cap);
  *races += b.races;
  *drains += b.drains;
  count_outcomes<POL>(P, S, cap, rollbacks, kept);
  const uint32_t st = a.words[11];  // status: after t (2 words) and nine counters
  *ties += (st & ST_TIE) ? 1 : 0;
  *unresolved += (st & ST_TIE_UNRESOLVED) ? 1 : 0;
  if (b.words[11] & ST_RACE_REDO) {  // the kernel discards this run; the eager pass redoes it
    ++*redo;
    return true;
  }
  if (a.words != b.words || a.head.h != b.head.h || a.head.ra != b.head.ra) {
    for (int i = 0; i < CK_WORDS; ++i)
      if (a.words[i] != b.words[i]) {
        fprintf(stderr, "MISMATCH alpha=%g delta=%g dmax=%g pol=%d ep=%llu: word %d eager %u deferred %u\n",
                cf.alpha, cf.delta, cf.dmax, POL, (unsigned long long)ep, i, a.words[i], b.words[i]);
        break;
      }
    return false;
  }
  return true;
}

int main(int argc, char** argv) {
  const int eps = argc > 1 ? atoi(argv[1]) : 100;
  const int steps = argc > 2 ? atoi(argv[2]) : 600;
  std::vector<Cfg> cfgs;
  for (double a : {0.05, 0.25, 0.33, 0.45, 0.5}) {
    cfgs.push_back(Cfg{a, 1e-9, 1e-9, 0, steps});        // the gym's gamma = .5 network
    cfgs.push_back(Cfg{a, 1e-9, 0.5e-9 / 0.3, 0, steps});  // gamma = .3: many redo flags
    cfgs.push_back(Cfg{a, 1e-13, 1e-13, 0, steps});      // same-instant ties are common
    cfgs.push_back(Cfg{a, 1e-9, 0.3e-9, 0, steps});      // releases always win
  }
  long n = 0, bad = 0, races = 0, drains = 0, rollbacks = 0, kept = 0, ties = 0, unresolved = 0;
  long redo = 0, redo_win = 0;  // episodes flagged; of them in the releases-always-win configs
  for (size_t c = 0; c < cfgs.size(); ++c)
    for (int pol = 0; pol < 4; ++pol)
      for (int e = 0; e < eps; ++e) {
        Cfg cf = cfgs[c];
        cf.policy = pol;
        bool ok = true;
        const long r0 = redo;
        switch (pol) {
          case 0: ok = compare<0>(cf, e, &races, &drains, &rollbacks, &kept, &ties, &unresolved, &redo); break;
          case 1: ok = compare<1>(cf, e, &races, &drains, &rollbacks, &kept, &ties, &unresolved, &redo); break;
          case 2: ok = compare<2>(cf, e, &races, &drains, &rollbacks, &kept, &ties, &unresolved, &redo); break;
          default: ok = compare<3>(cf, e, &races, &drains, &rollbacks, &kept, &ties, &unresolved, &redo); break;
        }
        if (c % 4 == 3) redo_win += redo - r0;
        ++n;
        bad += ok ? 0 : 1;
      }
  // emulated waves of 8 lanes, 6 list entries per lane
  long wave_eps = 0, wave_bad = 0, wave_drains = 0;
  for (const Cfg& c0 : cfgs) {
    NakParams P{};
    P.t_att = oracle::alpha_threshold(c0.alpha);
    P.d = 2;
    P.ev = 1.0;
    P.delta = c0.delta;
    P.dmax = c0.dmax;
    P.arrive = 1;
    P.max_steps = c0.steps;
    P.max_progress = __builtin_inf();
    P.max_time = __builtin_inf();
    P.cap = c0.steps + 64;
    for (int w = 0; w < (eps + 7) / 8; ++w) {
      P.policy = 2;
      wave_bad += run_wave<2>(P, 1000 + 8 * w, 8, 6, &wave_drains);
      P.policy = 3;
      wave_bad += run_wave<3>(P, 1000 + 8 * w, 8, 6, &wave_drains);
      wave_eps += 16;
    }
  }
  printf("{\"episodes\": %ld, \"mismatches\": %ld, \"races\": %ld, \"drains\": %ld, "
         "\"redo_flags\": %ld, \"ties_kept\": %ld, \"tie_episodes\": %ld, \"unresolved_episodes\": %ld, "
         "\"redo_episodes\": %ld, \"redo_episodes_release_wins\": %ld, "
         "\"wave_episodes\": %ld, \"wave_mismatches\": %ld, \"wave_drains\": %ld}\n",
         n, bad, races, drains, rollbacks, kept, ties, unresolved, redo, redo_win, wave_eps, wave_bad,
         wave_drains);
  return bad || wave_bad || redo_win ? 1 : 0;
}

// TEST INFRASTRUCTURE ONLY — CPU oracle, B_k part. See bk.h for the map to the reference
// sources.
#include "bk.h"

#include <algorithm>
#include <cmath>
#include <stdexcept>

#include "ocaml_sort.h"

namespace oracle {

static inline bool is_vote(const Block* b) { return b->value.kind == 1; }
static inline bool is_block(const Block* b) { return b->value.kind == 0; }

static int compare_pow(const Pow& a, const Pow& b) { return a < b ? -1 : (a > b ? 1 : 0); }

// bk.ml:110-132 (referee: global view, all parents)
bool bk_validity(const Block* b, int k) {
  if (is_vote(b)) {
    if (b->parents.size() != 1) return false;
    const Block* p = b->parents[0];
    return b->has_pow && is_block(p) && b->value.height == p->value.height;
  }
  if (b->parents.size() < 2) return false;
  const Block* pblock = b->parents[0];
  const Block* vote0 = b->parents[1];
  if (!(is_block(pblock) && is_vote(vote0))) return false;
  if (!vote0->has_pow) throw std::runtime_error("Option.get: vote without pow");
  bool ok = true;
  Pow h = bk_pow(vote0);
  int i = 1;
  for (size_t j = 2; j < b->parents.size(); ++j) {
    const Block* n = b->parents[j];
    if (!n->has_pow) throw std::runtime_error("Option.get: quorum member without pow");
    const Pow h2 = bk_pow(n);
    ok = is_vote(n) && compare_pow(h2, h) > 0 && ok;
    h = h2;
    ++i;
  }
  return pblock->value.height + 1 == b->value.height && i == k && ok &&
         b->signature == vote0->value.miner;
}

// bk.ml:151-176
void bk_reward(const Block* x, int scheme, int k, std::vector<double>& r) {
  if (!is_block(x)) return;
  if (scheme == BK_BLOCK) {
    if (x->signature >= 0) r[x->signature] += (double)k;
    return;
  }
  for (auto* y : x->parents)
    if (is_vote(y)) r[y->value.miner] += 1.;
}

// ---------------------------------------------------------------- Honest (bk.ml:185-311)

bool BkView::keep(const Block* b, int vf) const {
  switch (vf) {
    case VF_MINE: return b->vis[view].kind == WITHHELD || b->vis[view].kind == RELEASED;
    case VF_PUBLIC: return b->vis[view].kind == RELEASED || b->vis[view].kind == RECEIVED;
    default: return true;
  }
}

std::vector<Block*> BkView::children(const Block* b) const {
  std::vector<Block*> r;
  for (auto it = b->children_app.rbegin(); it != b->children_app.rend(); ++it)
    if (visible(*it)) r.push_back(*it);
  return r;
}

Block* BkView::last_block(Block* x) const {
  if (is_block(x)) return x;
  std::vector<Block*> p;
  for (auto* q : x->parents)
    if (visible(q)) p.push_back(q);
  if (p.size() != 1) throw std::runtime_error("invalid_dag: last block hits root");
  return p[0];
}

Pow BkView::leader_hash(const Block* x) const {
  if (!is_block(x)) throw std::invalid_argument("not a block");
  std::vector<const Block*> p;
  for (auto* q : x->parents)
    if (visible(q)) p.push_back(q);
  if (p.size() >= 2) {
    if (!p[1]->has_pow) throw std::invalid_argument("invalid dag / vote");
    return bk_pow(p[1]);
  }
  return bk_max_pow();  // genesis
}

int BkView::confirming(const Block* b, int vf) const {
  if (!is_block(b)) throw std::runtime_error("assert: confirming_votes of a vote");
  int n = 0;
  for (auto* c : children(b))
    if (is_vote(c) && keep(c, vf)) ++n;
  return n;
}

int BkView::compare_blocks(int vf, Block* a, Block* b) const {
  if (a == b) return 0;  // skip_eq Block.eq
  if (!is_block(a) || !is_block(b)) throw std::runtime_error("block_height_exn: not a block");
  if (a->value.height != b->value.height) return a->value.height < b->value.height ? -1 : 1;
  const int ca = confirming(a, vf), cb = confirming(b, vf);
  if (ca != cb) return ca < cb ? -1 : 1;
  const int c = compare_pow(leader_hash(b), leader_hash(a));  // neg compare_pow
  if (c != 0) return c;
  return float_compare(b->vis[view].time, a->vis[view].time);  // neg float visible_since
}

Block* BkView::update_head(int vf, Block* old, Block* consider) const {
  if (!is_block(consider)) throw std::runtime_error("assert: update_head with a vote");
  return compare_blocks(vf, consider, old) > 0 ? consider : old;
}

bool BkView::quorum(int vf, Block* b, std::vector<Block*>* q) const {
  Pow my_hash = bk_max_pow(), replace_hash = bk_max_pow();
  std::vector<Block*> mine, theirs;  // OCaml lists built by prepending: head = back()
  int nmine = 0, ntheirs = 0;
  for (auto* x : children(b)) {
    if (!is_vote(x) || !keep(x, vf)) continue;  // confirming_votes b |> List.filter vf
    if (x->value.miner == view) {
      my_hash = std::min(my_hash, bk_pow(x));
      mine.push_back(x);
      ++nmine;
    } else {
      theirs.push_back(x);
      ++ntheirs;
    }
  }
  if (replace_hash <= my_hash || nmine + ntheirs < k) return false;  // fast path
  auto by_pow = [](Block* x, Block* y) { return compare_pow(bk_pow(x), bk_pow(y)); };
  if (nmine >= k) {
    // Compare.first (by compare_pow) k mine; Array.of_list mine = list order = reversed push
    std::vector<Block*> a(mine.rbegin(), mine.rend());
    ocaml_array_sort(a, by_pow);
    q->assign(a.begin(), a.begin() + k);
    return true;
  }
  // fold over `theirs` (list order: reversed push order), prepending when hash > my_hash
  std::vector<Block*> th2;  // push order of the new prepends: head = back()
  for (auto it = theirs.rbegin(); it != theirs.rend(); ++it)
    if (bk_pow(*it) > my_hash) th2.push_back(*it);
  const int n2 = (int)th2.size();
  if (n2 < k - nmine) return false;  // fast path
  std::vector<Block*> a(th2.rbegin(), th2.rend());
  const int v = view;
  ocaml_array_sort(a, [v](Block* x, Block* y) {
    return float_compare(x->vis[v].time, y->vis[v].time);
  });
  std::vector<Block*> all(mine.rbegin(), mine.rend());  // mine @ theirs
  all.insert(all.end(), a.begin(), a.begin() + (k - nmine));
  // List.sort (stable merge sort); pow hashes are unique, so any sort agrees
  std::stable_sort(all.begin(), all.end(), [](Block* x, Block* y) { return bk_pow(x) < bk_pow(y); });
  *q = all;
  return true;
}

bool BkView::propose(int vf, Block* b, Draft* d) const {
  std::vector<Block*> q;
  if (!quorum(vf, b, &q)) return false;
  d->parents.clear();
  d->parents.push_back(b);
  d->parents.insert(d->parents.end(), q.begin(), q.end());
  d->data = NakData{b->value.height + 1, -1, 0, 0};
  d->sign = true;
  return true;
}

Draft BkView::puzzle_payload(Block* preferred) const {
  if (!is_block(preferred)) throw std::runtime_error("block_height_exn: not a block");
  Draft d;
  d.parents = {preferred};
  d.sign = false;
  d.data = NakData{preferred->value.height, view, 0, 1};
  return d;
}

Draft BkHonest::puzzle_payload() { return BkView{sim, id, sim->bk_k}.puzzle_payload(state); }

// bk.ml:297-310
Action BkHonest::handler(Kind, Block* x) {
  BkView V{sim, id, sim->bk_k};
  Block* b = V.last_block(x);
  Action a;
  Draft d;
  if (V.propose(VF_ALL, b, &d)) a.append.push_back(d);
  if (x->vis[id].kind == WITHHELD) a.share.push_back(x);
  state = V.update_head(VF_ALL, state, b);
  return a;
}

// bk.ml:134-147: global view, confirming votes counted over the whole DAG
Block* bk_winner(const std::vector<Block*>& l) {
  if (l.empty()) throw std::runtime_error("bk.winner: empty list");
  auto nconf = [](const Block* b) {
    int n = 0;
    for (auto* c : b->children_app) n += is_vote(c) ? 1 : 0;
    return n;
  };
  auto cmp = [&](Block* a, Block* b) {
    if (a == b) return 0;
    if (!is_block(a) || !is_block(b)) throw std::runtime_error("block_height_exn: not a block");
    if (a->value.height != b->value.height) return a->value.height < b->value.height ? -1 : 1;
    const int na = nconf(a), nb = nconf(b);
    return na < nb ? -1 : (na > nb ? 1 : 0);
  };
  Block* acc = l[0];
  for (size_t i = 1; i < l.size(); ++i)
    if (cmp(l[i], acc) > 0) acc = l[i];
  return acc;
}

// ---------------------------------------------------------------- policies / observation

// bk_ssz.ml:346-401
int bk_policy(int policy, const BkObs& o, int k, const BkTable* table) {
  const int h = o.public_blocks, a = o.private_blocks;
  switch (policy) {
    case BKPOL_HONEST: return h > a ? ADOPT_PROCEED : OVERRIDE_PROCEED;
    case BKPOL_GET_AHEAD:
      if (h > a) return ADOPT_PROCEED;
      if (h < a) return OVERRIDE_PROCEED;
      return WAIT_PROCEED;
    case BKPOL_MINOR_DELAY:
      if (h > a) return ADOPT_PROCEED;
      if (h == 0) return WAIT_PROCEED;
      return OVERRIDE_PROCEED;
    case BKPOL_AVOID_LOSS: {
      const int hp = h * k + o.public_votes, ap = a * k + o.private_votes_inclusive;
      if (h == 0) return WAIT_PROCEED;
      if (h == 1 && hp == ap) return MATCH_PROCEED;
      if (hp > ap) return ADOPT_PROCEED;
      if (hp == ap - 1) return OVERRIDE_PROCEED;
      if (h < a - 10) return OVERRIDE_PROCEED;
      return WAIT_PROCEED;
    }
    case BKPOL_TABLE: {
      const int D = table->dim, K1 = table->k + 1;
      auto cl = [](int x, int hi) { return std::min(std::max(x, 0), hi); };
      const int64_t idx =
          ((((int64_t)cl(h, D - 1) * D + cl(a, D - 1)) * K1 + cl(o.public_votes, K1 - 1)) * K1 +
           cl(o.private_votes_inclusive, K1 - 1)) * 3 + o.event;
      return table->actions[idx];
    }
  }
  throw std::invalid_argument("unknown policy");
}

// ssz_tools.ml:1-74 NormalizeObs with bk_ssz.ml:37-48 normalizers
void bk_obs_to_floats(const BkObs& o, bool unit, int k, double out[BK_OBS_LEN]) {
  const int v[BK_OBS_LEN] = {o.public_blocks,           o.private_blocks, o.diff_blocks,
                             o.public_votes,            o.private_votes_inclusive,
                             o.private_votes_exclusive, o.lead,           o.event};
  for (int i = 0; i < BK_OBS_LEN; ++i) {
    if (i == 6) {
      out[i] = v[i] ? 1. : 0.;  // Bool
    } else if (i == 7) {
      out[i] = unit ? (double)v[i] / 2. : (double)v[i];  // Discrete, 3 values
    } else if (!unit) {
      out[i] = (double)v[i];
    } else {
      const double scale = (i >= 3) ? (double)k : 1.;
      if (i == 2)
        out[i] = 0.5 + (1. / M_PI * std::atan((double)v[i] / scale));
      else
        out[i] = 2. / M_PI * std::atan((double)v[i] / scale);
    }
  }
}

BkObs bk_obs_of_floats(const double in[BK_OBS_LEN], bool unit, int k) {
  int v[BK_OBS_LEN];
  for (int i = 0; i < BK_OBS_LEN; ++i) {
    if (i == 6) {
      v[i] = in[i] >= 0.5 ? 1 : 0;
    } else if (i == 7) {
      v[i] = unit ? (int)std::floor(in[i] * 2.) : (int)in[i];
    } else if (!unit) {
      v[i] = (int)in[i];
    } else {
      const double scale = (i >= 3) ? (double)k : 1.;
      if (i == 2)
        v[i] = (int)std::round(std::tan(M_PI * (in[i] - 0.5)) * scale);
      else
        v[i] = (int)std::round(std::tan(M_PI / 2. * in[i]) * scale);
    }
  }
  return BkObs{v[0], v[1], v[2], v[3], v[4], v[5], v[6], v[7]};
}

// ssz_tools.ml:64-74 range; bk_ssz.ml:52-74
void bk_obs_range(bool unit, double low[BK_OBS_LEN], double high[BK_OBS_LEN]) {
  for (int i = 0; i < BK_OBS_LEN; ++i) {
    if (unit) {
      low[i] = 0.;
      high[i] = 1.;
    } else if (i == 2) {
      low[i] = -1. / 0.;
      high[i] = 1. / 0.;
    } else if (i == 6) {
      low[i] = 0.;
      high[i] = 0.;  // Bool range is (0, 0) in the reference
    } else if (i == 7) {
      low[i] = 0.;
      high[i] = 2.;
    } else {
      low[i] = 0.;
      high[i] = 1. / 0.;
    }
  }
}

// ---------------------------------------------------------------- agent (bk_ssz.ml:148-332)

// bk_ssz.ml:196-221
void BkSszAgent::prepare(Kind kd, Block* x) {
  const BkView v = V();
  Block* p = pub;
  for (auto* m : pending) p = v.update_head(VF_PUBLIC, p, v.last_block(m));
  Block* q = priv;
  switch (kd) {
    case K_APPEND:
      q = x;
      o_event = 0;
      break;
    case K_POW: o_event = 1; break;
    case K_NETWORK:
      p = v.update_head(VF_PUBLIC, p, v.last_block(x));
      o_event = 2;
      break;
  }
  o_pub = p;
  o_priv = q;
  o_common = common_ancestor(*sim, my_id, p, q);
  if (!o_common) throw std::runtime_error("Option.get: no common ancestor");
}

// bk_ssz.ml:225-263
BkObs BkSszAgent::observe() const {
  const BkView v = V();
  BkObs o;
  o.public_votes = 0;
  std::vector<Block*> pub_votes;
  for (auto* c : v.children(o_pub)) {
    if (!is_vote(c)) continue;
    pub_votes.push_back(c);
    if (v.keep(c, VF_PUBLIC)) ++o.public_votes;
  }
  o.private_votes_inclusive = o.private_votes_exclusive = 0;
  for (auto* c : v.children(o_priv)) {
    if (!is_vote(c)) continue;
    ++o.private_votes_inclusive;
    if (v.keep(c, VF_MINE)) ++o.private_votes_exclusive;
  }
  o.lead = 0;
  if (!pub_votes.empty()) {
    std::vector<Block*> a = pub_votes;
    ocaml_array_sort(a, [](Block* x, Block* y) { return compare_pow(bk_pow(x), bk_pow(y)); });
    o.lead = a[0]->signature == my_id ? 1 : 0;  // votes are unsigned: always false
  }
  const int ca = v.last_block(o_common)->value.height;
  const int ph = o_priv->value.height, qh = o_pub->value.height;
  o.private_blocks = ph - ca;
  o.public_blocks = qh - ca;
  o.diff_blocks = ph - qh;
  o.event = o_event;
  return o;
}

// bk_ssz.ml:265-331
Action BkSszAgent::apply(int action) {
  if (action < 0 || action >= BK_N_ACTIONS)
    throw std::invalid_argument("index out of bounds");
  const BkView v = V();
  const int vw = my_id;
  auto release = [&](bool override_) {
    int height = o_pub->value.height;
    int nvotes = 0;
    for (auto* c : v.children(o_pub))
      if (is_vote(c) && v.keep(c, VF_PUBLIC)) ++nvotes;
    if (override_) {
      if (nvotes >= k) {
        height = height + 1;
        nvotes = 0;
      } else {
        nvotes = nvotes + 1;
      }
    }
    Block* block = o_priv;
    while (block->value.height > height) {
      std::vector<Block*> ps;
      for (auto* q : block->parents)
        if (v.visible(q)) ps.push_back(q);
      if (ps.empty() || !is_block(ps[0])) throw std::runtime_error("Option.get: parent_block");
      block = ps[0];
    }
    if (nvotes >= k) {
      for (auto* c : v.children(block))
        if (is_block(c)) {
          block = c;
          nvotes = 0;
          break;
        }
    }
    std::vector<Block*> votes;
    for (auto* c : v.children(block))
      if (is_vote(c)) votes.push_back(c);
    std::vector<Block*> share{block};
    if ((int)votes.size() >= nvotes) {
      std::vector<Block*> a = votes;
      ocaml_array_sort(a, [vw](Block* x, Block* y) {
        return float_compare(x->vis[vw].time, y->vis[vw].time);
      });
      share.insert(share.end(), a.begin(), a.begin() + nvotes);
    } else {
      share.insert(share.end(), votes.begin(), votes.end());
    }
    return share;
  };
  Action a;
  Block* np = o_priv;
  switch (action % 4) {
    case 0: np = o_pub; break;                // Adopt
    case 1: a.share = release(true); break;   // Override
    case 2: a.share = release(false); break;  // Match
    default: break;                           // Wait
  }
  const int vf = action >= 4 ? VF_ALL : VF_MINE;  // Proceed: Inclusive, Prolong: Exclusive
  Draft d;
  if (v.propose(vf, np, &d)) a.append.push_back(d);
  pub = o_pub;
  priv = np;
  pending = a.share;
  return a;
}

Action BkSszAttackerNode::handler(Kind kd, Block* b) {
  agent.prepare(kd, b);
  const int act = policy == BKPOL_RANDOM ? agent.sim->rng->rand_action(nrand++, 8)
                                         : bk_policy(policy, agent.observe(), agent.k, table);
  return agent.apply(act);
}

// ---------------------------------------------------------------- gym engine

GymBk::GymBk(const GymParams& p_, int k_, int scheme_, int mode, OcamlRandom* oc, uint64_t seed_,
             uint64_t ep)
    : p(p_), k(k_), scheme(scheme_), rng_mode(mode), ocaml(oc), seed(seed_), episode(ep) {
  std::string e = gym_params_error(p);
  if (!e.empty()) throw std::invalid_argument(e);
  if (k < 1) throw std::invalid_argument("k must be positive");
  net = Network::selfish_mining(p.alpha, p.activation_delay, p.gamma, p.propagation_delay,
                                p.defenders);
}

// engine.ml:108-121
Kind GymBk::skip_to_interaction(Block** blk) {
  Event ev;
  for (;;) {
    if (!sim->dequeue(&ev)) throw std::runtime_error("simulation should continue forever");
    if (ev.type == EV_ONNODE && ev.node == 0) {
      *blk = ev.blk;
      return ev.kind;
    }
    if (ev.type == EV_DAG && ev.node == 0 && ev.kind == K_POW) {
      Draft d = agent.puzzle_payload();
      Block* v = sim->append(true, 0, d);
      sim->schedule_now(Event{EV_MAKEVIS, 0, K_POW, v, -1});
      continue;
    }
    sim->handle_event(ev);
  }
}

static std::unique_ptr<SimRng> make_bk_rng(int rng_mode, OcamlRandom* oc, uint64_t seed,
                                           uint64_t ep, const Network& net) {
  if (rng_mode == 0)
    return trace_wrap(std::unique_ptr<SimRng>(new OcamlSimRng(oc, net)), net, true);
  auto* r = new KeyedSimRng(seed, ep, net, needs_general_weights(net));
  r->serial_links = true;
  return trace_wrap(std::unique_ptr<SimRng>(r), net, true);
}

void GymBk::init() {
  rng = make_bk_rng(rng_mode, ocaml, seed, episode, net);
  sim.reset(new Sim(net, rng.get()));
  sim->proto = 2;
  sim->bk_k = k;
  sim->bk_scheme = scheme;
  std::vector<std::unique_ptr<NodeImpl>> nodes;
  const int n = (int)net.nodes.size();
  for (int i = 0; i < n; i++) {
    if (i == 0)
      nodes.emplace_back(new DummyNode());
    else
      nodes.emplace_back(new BkHonest());
  }
  sim->init(std::move(nodes));
  Block* root = sim->roots.back();
  static_cast<DummyNode*>(sim->nodes[0].get())->state = root;
  for (int i = 1; i < n; i++) static_cast<BkHonest*>(sim->nodes[i].get())->state = root;
  agent = BkSszAgent();
  agent.sim = sim.get();
  agent.my_id = 0;
  agent.k = k;
  agent.init(root);
  Block* b;
  Kind kd = skip_to_interaction(&b);
  agent.prepare(kd, b);
  episode_steps = 0;
  last_progress = last_chain_time = last_sim_time = last_reward_attacker =
      last_reward_defender = 0.;
}

void GymBk::observe(double obs[BK_OBS_LEN]) const {
  bk_obs_to_floats(agent.observe(), p.unit_obs, k, obs);
}

void GymBk::reset(double obs[BK_OBS_LEN]) {
  init();
  observe(obs);
}

// engine.ml:176-249
double GymBk::step(int action, double obs[BK_OBS_LEN], bool* done, StepInfo* info) {
  Action act = agent.apply(action);
  sim->handle_action(0, act);
  episode_steps++;
  Block* b;
  Kind kd = skip_to_interaction(&b);
  Block* attacker_pref = agent.priv;
  agent.prepare(kd, b);
  std::vector<Block*> prefs;
  prefs.push_back(attacker_pref);
  for (int i = 1; i < sim->n_nodes; i++) prefs.push_back(sim->nodes[i]->preferred());
  Block* head = bk_winner(prefs);
  const double progress = sim->progress(head);
  *done = !(episode_steps < p.max_steps && progress < p.max_progress && sim->now < p.max_time);
  double ra = 0., rd = 0.;
  for (int i = 0; i < sim->n_nodes; i++) {
    if (i == 0)
      ra += head->rewards[i];
    else
      rd += head->rewards[i];
  }
  const double chain_time = Sim::timestamp(head);
  const double sim_time = sim->now;
  const double reward = ra - last_reward_attacker;
  if (info) {
    info->step_reward_attacker = ra - last_reward_attacker;
    info->step_reward_defender = rd - last_reward_defender;
    info->step_progress = progress - last_progress;
    info->step_chain_time = chain_time - last_chain_time;
    info->step_sim_time = sim_time - last_sim_time;
    info->episode_reward_attacker = ra;
    info->episode_reward_defender = rd;
    info->episode_progress = progress;
    info->episode_chain_time = chain_time;
    info->episode_sim_time = sim_time;
    info->episode_n_steps = episode_steps;
    info->episode_n_activations = sim->c_activations;
    info->head_height = head->value.height;
    info->head_miner = head->signature;  // B_k: the head's signer (leader); -1 for genesis
    info->head_work = 0;
  }
  last_chain_time = chain_time;
  last_sim_time = sim_time;
  last_reward_attacker = ra;
  last_reward_defender = rd;
  last_progress = progress;
  observe(obs);
  return reward;
}

void bk_loop_task(const Network& net, int rng_mode, OcamlRandom* r, uint64_t seed,
                  uint64_t episode, int k, int scheme, int policy, const BkTable* table,
                  int activations, BkLoopResult* out) {
  std::unique_ptr<SimRng> rng = make_bk_rng(rng_mode, r, seed, episode, net);
  Sim sim(net, rng.get());
  sim.proto = 2;
  sim.bk_k = k;
  sim.bk_scheme = scheme;
  sim.zt_limit = 4096;
  const int n = (int)net.nodes.size();
  std::vector<std::unique_ptr<NodeImpl>> nodes;
  BkSszAttackerNode* att = nullptr;
  for (int i = 0; i < n; ++i) {
    if (i == 0 && policy >= 0) {
      att = new BkSszAttackerNode();
      att->policy = policy;
      att->table = table;
      nodes.emplace_back(att);
    } else {
      nodes.emplace_back(new BkHonest());
    }
  }
  sim.init(std::move(nodes));
  Block* root = sim.roots.back();
  for (int i = 0; i < n; ++i) {
    if (i == 0 && att) {
      att->agent.sim = &sim;
      att->agent.my_id = 0;
      att->agent.k = k;
      att->agent.init(root);
    } else {
      static_cast<BkHonest*>(sim.nodes[i].get())->state = root;
    }
  }
  sim.loop(activations);
  std::vector<Block*> prefs;
  for (auto& nd : sim.nodes) prefs.push_back(nd->preferred());
  Block* h = bk_winner(prefs);
  out->activations.assign(sim.activations.begin(), sim.activations.end());
  out->rewards = h->rewards;
  out->head_time = Sim::timestamp(h);
  out->head_progress = sim.progress(h);
  out->head_height = h->value.height;
  out->head_signer = h->signature;
  out->n_vertices = (int64_t)sim.dag.size();
}

}  // namespace oracle

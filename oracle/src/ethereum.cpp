// TEST INFRASTRUCTURE ONLY — CPU oracle, Ethereum part. See ethereum.h for the map to
// the reference sources.
#include "ethereum.h"

#include <algorithm>
#include <cmath>
#include <stdexcept>

#include "ocaml_sort.h"

namespace oracle {

static std::vector<Block*> parents_in(const Sim& sim, int view, const Block* b) {
  std::vector<Block*> r;
  for (auto* p : b->parents)
    if (sim.visible(view, p)) r.push_back(p);
  return r;
}

static bool contains(const std::vector<Block*>& l, const Block* x) {
  return std::find(l.begin(), l.end(), x) != l.end();
}

// ethereum.ml:102-151 (global view: all parents)
bool eth_validity(const Block* b) {
  if (!b->has_pow || b->parents.empty()) return false;
  const Block* p = b->parents[0];
  std::vector<Block*> uncles(b->parents.begin() + 1, b->parents.end());
  // ancestors: p and up to six generations above it (or the root); previous uncles:
  // the uncles those blocks include
  std::vector<const Block*> ancestors, previous_uncles;
  {
    const Block* x = p;
    for (int gen = 0; gen <= 6; ++gen) {
      ancestors.push_back(x);
      if (x->parents.empty()) break;
      for (size_t i = 1; i < x->parents.size(); ++i) previous_uncles.push_back(x->parents[i]);
      x = x->parents[0];
    }
  }
  auto in = [](const std::vector<const Block*>& l, const Block* x) {
    return std::find(l.begin(), l.end(), x) != l.end();
  };
  const auto& bd = b->value;
  const auto& pd = p->value;
  if (bd.height != pd.height + 1) return false;
  if (bd.work != pd.work + 1 + (int)uncles.size()) return false;
  if (bd.miner < 0) return false;
  if (uncles.size() > 2) return false;
  for (auto* u : uncles) {
    const int k = bd.height - u->value.height;
    if (!(1 <= k && k <= 6)) return false;
    int n = 0;
    for (auto* q : b->parents) n += q == u;
    if (n != 1) return false;
    if (u->parents.empty() || !in(ancestors, u->parents[0])) return false;
    if (in(ancestors, u) || in(previous_uncles, u)) return false;
  }
  return true;
}

// ethereum.ml:173-197; base_reward = 1
void eth_reward(const Block* x, int scheme, std::vector<double>& r) {
  const int n_uncles = (int)x->parents.size() - 1;
  if (x->value.miner >= 0) r[x->value.miner] += 1. + ((double)n_uncles * 0.03125 * 1.);
  for (int i = 1; i <= n_uncles; ++i) {
    const Block* u = x->parents[i];
    if (u->value.miner < 0) continue;
    if (scheme == 0)
      r[u->value.miner] += 0.9375 * 1.;
    else {
      const double delta = (double)(x->value.height - u->value.height);
      r[u->value.miner] += (8. - delta) / 8. * 1.;
    }
  }
}

// ethereum.ml:234-277
Draft eth_payload(const Sim& sim, int view, Block* preferred,
                  const std::function<bool(Block*)>& uncle_filter) {
  std::vector<Block*> nua;  // non-uncle ancestors, generation 1..6 (gen 1 first)
  std::vector<Block*> in_chain{preferred};
  {
    Block* b = preferred;
    int gen = 0;
    for (;;) {
      std::vector<Block*> p = parents_in(sim, view, b);
      if (p.empty()) break;
      ++gen;
      if (gen > 6) break;
      nua.push_back(p[0]);
      in_chain.insert(in_chain.end(), p.begin(), p.end());
      b = p[0];
    }
  }
  // fold_left over [gen6; ...; gen1] prepending: uncles(gen1) @ ... @ uncles(gen6)
  std::vector<Block*> cands;
  for (Block* b : nua) {
    // Dag children list is newest first (dag.ml:32)
    for (auto it = b->children_app.rbegin(); it != b->children_app.rend(); ++it) {
      Block* c = *it;
      if (!sim.visible(view, c)) continue;
      if (contains(in_chain, c)) continue;
      std::vector<Block*> cp = parents_in(sim, view, c);
      if (cp.empty() || !contains(nua, cp[0])) continue;
      cands.push_back(c);
    }
  }
  std::vector<Block*> filtered;
  for (Block* c : cands)
    if (uncle_filter(c)) filtered.push_back(c);
  // uncle_preference: by (not appended_by_me, height) ascending (ethereum.ml:226-232)
  auto cmp = [view](Block* x, Block* y) {
    const int bx = eth_appended_by(x, view) ? 0 : 1, by = eth_appended_by(y, view) ? 0 : 1;
    if (bx != by) return bx < by ? -1 : 1;
    const int hx = x->value.height, hy = y->value.height;
    return hx < hy ? -1 : (hx > hy ? 1 : 0);
  };
  std::vector<Block*> uncles = ocaml_at_most_first(filtered, cmp, 2);
  Draft d;
  d.parents.push_back(preferred);
  d.parents.insert(d.parents.end(), uncles.begin(), uncles.end());
  d.data.height = preferred->value.height + 1;
  d.data.work = preferred->value.work + 1 + (int)uncles.size();
  d.data.miner = view;
  d.sign = false;
  return d;
}

Draft EthHonest::puzzle_payload() {
  return eth_payload(*sim, id, state, [](Block*) { return true; });
}

// ethereum.ml:279-297
Action EthHonest::handler(Kind k, Block* v) {
  if (k == K_APPEND) throw std::runtime_error("not implemented");
  Action a;
  if (v->value.height > state->value.height) state = v;
  if (v->vis[id].kind == WITHHELD) a.share = {v};
  return a;
}

// ---------------------------------------------------------------- attack space

static bool mining_filter(bool own, bool foreign, const Block* x, int view) {
  const bool mine = eth_appended_by(x, view);
  return (own && mine) || (foreign && !mine);
}

Draft EthSszAgent::puzzle_payload() const {
  const bool o = own, f = foreign;
  const int v = my_id;
  return eth_payload(*sim, my_id, priv,
                     [o, f, v](Block* x) { return mining_filter(o, f, x, v); });
}

// ethereum_ssz.ml:325-362
void EthSszAgent::prepare(Kind k, Block* x) {
  Block* p = pub;
  for (auto* m : pending)
    if (m->value.height > p->value.height) p = m;
  Block* q = priv;
  switch (k) {
    case K_APPEND: throw std::runtime_error("not implemented");
    case K_NETWORK:
      if (x->value.height > p->value.height) p = x;
      o_event = 1;
      break;
    case K_POW:
      q = x;
      o_event = 0;
      break;
  }
  o_pub = p;
  o_priv = q;
  o_common = common_ancestor(*sim, my_id, p, q);
  if (!o_common) throw std::runtime_error("Option.get: no common ancestor");
}

// ethereum_ssz.ml:364-396
EthObs EthSszAgent::observe() const {
  const auto& c = o_common->value;
  const auto& pr = o_priv->value;
  const auto& pu = o_pub->value;
  const int v = my_id;
  const Sim& s = *sim;
  EthObs o;
  o.public_height = pu.height - c.height;
  o.public_work = pu.work - c.work;
  o.public_orphans =
      (int)eth_payload(s, v, o_pub,
                       [v](Block* x) {
                         return x->vis[v].kind == RELEASED || x->vis[v].kind == RECEIVED;
                       })
          .parents.size() -
      1;
  o.private_height = pr.height - c.height;
  o.private_work = pr.work - c.work;
  o.private_orphans_inclusive =
      (int)eth_payload(s, v, o_priv, [v](Block* x) { return mining_filter(true, true, x, v); })
          .parents.size() -
      1;
  o.private_orphans_exclusive =
      (int)eth_payload(s, v, o_priv, [v](Block* x) { return mining_filter(true, false, x, v); })
          .parents.size() -
      1;
  o.diff_height = o.private_height - o.public_height;
  o.diff_work = o.private_work - o.public_work;
  o.event = o_event;
  return o;
}

// ethereum_ssz.ml:398-429
Action EthSszAgent::apply(int index) {
  if (index < 0 || index >= ETH_N_ACTIONS)
    throw std::invalid_argument("Invalid_argument index out of bounds");
  const int action = index / 4;
  const bool m_own = (index & 2) != 0, m_foreign = (index & 1) != 0;
  auto release_upto = [&](int target) {
    Block* b = o_priv;
    while (b->value.height > target) {
      std::vector<Block*> p = parents_in(*sim, my_id, b);
      if (p.empty()) throw std::runtime_error("Option.get");
      b = p[0];
    }
    return b;
  };
  Action a;
  Block* np = o_priv;
  switch (action) {
    case ADOPT_RELEASE:
      a.share = {o_priv};
      np = o_pub;
      break;
    case ADOPT_DISCARD: np = o_pub; break;
    case E_MATCH: a.share = {release_upto(o_pub->value.height)}; break;
    case E_OVERRIDE: a.share = {release_upto(o_pub->value.height + 1)}; break;
    case RELEASE1: a.share = {release_upto(o_common->value.height + 1)}; break;
    case E_WAIT: break;
  }
  pub = o_pub;
  priv = np;
  pending = a.share;
  own = m_own;
  foreign = m_foreign;
  return a;
}

Action EthSszAttackerNode::handler(Kind k, Block* b) {
  agent.prepare(k, b);
  if (policy == ETH_POL_RANDOM) return agent.apply(agent.sim->rng->rand_action(nrand++, 24));
  return agent.apply(eth_policy(policy, agent.observe(), table));
}

int eth_policy(int policy, const EthObs& o, const EthTable* t) {
  if (policy != ETH_POL_TABLE) return eth_policy(policy, o);
  auto cl = [](int x, int hi) { return x < 0 ? 0 : (x > hi ? hi : x); };
  const int D = t->dim;
  return t->actions[(cl(o.public_height, D - 1) * D + cl(o.private_height, D - 1)) * 2 + o.event];
}

// ethereum_ssz.ml:444-521
int eth_policy(int policy, const EthObs& o) {
  switch (policy) {
    case EPOL_HONEST:
      return eth_action_index(o.public_work > 0 ? ADOPT_RELEASE : E_OVERRIDE, true, true);
    case EPOL_SELFISH_RELEASE:
    case EPOL_SELFISH_DISCARD: {
      // Byzantium preference is `HeaviestChain` -> compare work
      const int adopt = policy == EPOL_SELFISH_RELEASE ? ADOPT_RELEASE : ADOPT_DISCARD;
      const int pp = o.private_work, qp = o.public_work;
      int a;
      if (pp < qp)
        a = adopt;
      else if (pp == 0 && qp == 0)
        a = E_WAIT;
      else if (qp == 0)
        a = E_WAIT;
      else
        a = E_OVERRIDE;
      return eth_action_index(a, true, false);
    }
    case EPOL_FN19:
    case EPOL_FN19PKEL: {
      const bool pkel = policy == EPOL_FN19PKEL;
      const int ph = o.private_height, qh = o.public_height;
      int a;
      if (o.event == 0)
        a = (ph == 2 && qh == 1) ? E_OVERRIDE : E_WAIT;
      else if (ph < qh)
        a = pkel ? ADOPT_RELEASE : ADOPT_DISCARD;
      else if (ph == qh)
        a = E_MATCH;
      else if (ph == qh + 1)
        a = E_OVERRIDE;
      else
        a = RELEASE1;
      return eth_action_index(a, true, !pkel);
    }
  }
  throw std::invalid_argument("unknown ethereum policy");
}

// ssz_tools.ml NormalizeObs: UnboundedInt {non_negative; scale = 1}, Discrete event
void eth_obs_to_floats(const EthObs& o, bool unit, double out[ETH_OBS_LEN]) {
  const int v[ETH_OBS_LEN] = {o.public_height,  o.public_work,
                              o.private_height, o.private_work,
                              o.diff_height,    o.diff_work,
                              o.public_orphans, o.private_orphans_inclusive,
                              o.private_orphans_exclusive, o.event};
  for (int i = 0; i < ETH_OBS_LEN; ++i) {
    const bool signed_ = i == 4 || i == 5;
    if (!unit || i == 9)
      out[i] = (double)v[i] / 1.0;
    else if (signed_)
      out[i] = 0.5 + (1. / M_PI * std::atan((double)v[i] / 1.0));
    else
      out[i] = 2. / M_PI * std::atan((double)v[i] / 1.0);
  }
}

EthObs eth_obs_of_floats(const double in[ETH_OBS_LEN], bool unit) {
  int v[ETH_OBS_LEN];
  for (int i = 0; i < ETH_OBS_LEN; ++i) {
    const bool signed_ = i == 4 || i == 5;
    if (i == 9)
      v[i] = (int)std::floor(in[i] * 1.0);
    else if (!unit)
      v[i] = (int)in[i];
    else if (signed_)
      v[i] = (int)std::round(std::tan(M_PI * (in[i] - 0.5)) * 1.0);
    else
      v[i] = (int)std::round(std::tan(M_PI / 2. * in[i]) * 1.0);
  }
  return EthObs{v[0], v[1], v[2], v[3], v[4], v[5], v[6], v[7], v[8], v[9]};
}

// ---------------------------------------------------------------- gym engine

GymEthereum::GymEthereum(const GymParams& p_, int scheme_, int mode, OcamlRandom* oc,
                         uint64_t seed_, uint64_t ep)
    : p(p_), scheme(scheme_), rng_mode(mode), ocaml(oc), seed(seed_), episode(ep) {
  std::string e = gym_params_error(p);
  if (!e.empty()) throw std::invalid_argument(e);
  net = Network::selfish_mining(p.alpha, p.activation_delay, p.gamma, p.propagation_delay,
                                p.defenders);
}

// engine.ml:108-121
Kind GymEthereum::skip_to_interaction(Block** blk) {
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

void GymEthereum::init() {
  if (rng_mode == 0)
    rng.reset(new OcamlSimRng(ocaml, net));
  else
    rng.reset(new KeyedSimRng(seed, episode, net));
  rng = trace_wrap(std::move(rng), net, false);
  sim.reset(new Sim(net, rng.get()));
  sim->proto = 1;
  sim->eth_scheme = scheme;
  std::vector<std::unique_ptr<NodeImpl>> nodes;
  const int n = (int)net.nodes.size();
  for (int i = 0; i < n; i++) {
    if (i == 0)
      nodes.emplace_back(new DummyNode());
    else
      nodes.emplace_back(new EthHonest());
  }
  sim->init(std::move(nodes));
  Block* root = sim->roots.back();
  static_cast<DummyNode*>(sim->nodes[0].get())->state = root;
  for (int i = 1; i < n; i++) static_cast<EthHonest*>(sim->nodes[i].get())->state = root;
  agent = EthSszAgent();
  agent.sim = sim.get();
  agent.my_id = 0;
  agent.init(root);
  Block* b;
  Kind k = skip_to_interaction(&b);
  agent.prepare(k, b);
  episode_steps = 0;
  last_progress = last_chain_time = last_sim_time = last_reward_attacker =
      last_reward_defender = 0.;
}

void GymEthereum::observe(double obs[ETH_OBS_LEN]) const {
  eth_obs_to_floats(agent.observe(), p.unit_obs, obs);
}

void GymEthereum::reset(double obs[ETH_OBS_LEN]) {
  init();
  observe(obs);
}

// engine.ml:176-249
double GymEthereum::step(int action, double obs[ETH_OBS_LEN], bool* done, StepInfo* info) {
  Action act = agent.apply(action);
  sim->handle_action(0, act);
  episode_steps++;
  Block* b;
  Kind k = skip_to_interaction(&b);
  Block* attacker_pref = agent.priv;
  agent.prepare(k, b);
  std::vector<Block*> prefs;
  prefs.push_back(attacker_pref);
  for (int i = 1; i < sim->n_nodes; i++) prefs.push_back(sim->nodes[i]->preferred());
  Block* head = Sim::winner(prefs);
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
    info->head_miner = head->value.miner;
    info->head_work = head->value.work;
  }
  last_chain_time = chain_time;
  last_sim_time = sim_time;
  last_reward_attacker = ra;
  last_reward_defender = rd;
  last_progress = progress;
  observe(obs);
  return reward;
}

void eth_two_agents_task(int rng_mode, OcamlRandom* r, uint64_t seed, uint64_t episode,
                         double alpha, int scheme, int policy, int activations,
                         EthLoopResult* out, const EthTable* table) {
  Network net = Network::two_agents(1.0, alpha);
  std::unique_ptr<SimRng> rng;
  if (rng_mode == 0)
    rng.reset(new OcamlSimRng(r, net));
  else
    rng.reset(new KeyedSimRng(seed, episode, net));
  rng = trace_wrap(std::move(rng), net, false);
  Sim sim(net, rng.get());
  sim.proto = 1;
  sim.eth_scheme = scheme;
  std::vector<std::unique_ptr<NodeImpl>> nodes;
  auto* att = new EthSszAttackerNode();
  att->policy = policy;
  att->table = table;
  nodes.emplace_back(att);
  nodes.emplace_back(new EthHonest());
  sim.init(std::move(nodes));
  Block* root = sim.roots.back();
  att->agent.sim = &sim;
  att->agent.my_id = 0;
  att->agent.init(root);
  static_cast<EthHonest*>(sim.nodes[1].get())->state = root;
  sim.loop(activations);
  Block* h = sim.head();
  for (int i = 0; i < 2; i++) {
    out->activations[i] = sim.activations[i];
    out->rewards[i] = h->rewards[i];
  }
  out->head_time = Sim::timestamp(h);
  out->head_progress = sim.progress(h);
  out->head_height = h->value.height;
  out->head_work = h->value.work;
  out->diag = sim.diag;
}

}  // namespace oracle

// TEST INFRASTRUCTURE ONLY — CPU oracle. See des.h for the reference map.
#include "des.h"

#include <algorithm>
#include <cmath>
#include <set>
#include <stdexcept>

namespace oracle {

// ---------------------------------------------------------------- OrderedQueue

int float_compare(double a, double b) {
  // OCaml Float.compare: total order, nan equal to itself and below everything
  bool na = std::isnan(a), nb = std::isnan(b);
  if (na || nb) {
    if (na && nb) return 0;
    return na ? -1 : 1;
  }
  if (a < b) return -1;
  if (a > b) return 1;
  return 0;
}

int SkewHeap::alloc(double t, int ev) {
  int i;
  if (!freelist.empty()) {
    i = freelist.back();
    freelist.pop_back();
  } else {
    i = (int)pool.size();
    pool.push_back(N{});
  }
  pool[i] = N{t, ev, -1, -1};
  return i;
}

// orderedQueue.ml:17-26
int SkewHeap::ins(int node, double t, int ev) {
  if (node < 0) return alloc(t, ev);
  if (float_compare(t, pool[node].t) < 0) {
    // Node (time, evt, h this_time this_evt left, right)
    double ot = pool[node].t;
    int oe = pool[node].ev;
    int l = pool[node].l;
    pool[node].t = t;
    pool[node].ev = ev;
    int nl = ins(l, ot, oe);
    pool[node].l = nl;
    return node;
  }
  // Node (this_time, this_evt, h time evt right, left)
  int l = pool[node].l, r = pool[node].r;
  int nr = ins(r, t, ev);
  pool[node].l = nr;
  pool[node].r = l;
  return node;
}

// orderedQueue.ml:28-40
int SkewHeap::remove_top(int node) {
  int l = pool[node].l, r = pool[node].r;
  if (r < 0) {
    freelist.push_back(node);
    return l;
  }
  if (l < 0) {
    freelist.push_back(node);
    return r;
  }
  if (float_compare(pool[l].t, pool[r].t) <= 0) {
    pool[node].t = pool[l].t;
    pool[node].ev = pool[l].ev;
    int nl = remove_top(l);
    pool[node].l = nl;
  } else {
    pool[node].t = pool[r].t;
    pool[node].ev = pool[r].ev;
    int nr = remove_top(r);
    pool[node].r = nr;
  }
  return node;
}

bool SkewHeap::dequeue(double* t, int* ev) {
  if (root < 0) return false;
  *t = pool[root].t;
  *ev = pool[root].ev;
  root = remove_top(root);
  len--;
  return true;
}

// ---------------------------------------------------------------- Network

Network Network::two_agents(double activation_delay, double alpha) {
  Network n;
  n.flooding = false;
  n.activation_delay = activation_delay;
  n.nodes.resize(2);
  n.nodes[0].compute = alpha;
  n.nodes[0].links = {Link{1, D_CONST, 0.0, 0.0}};
  n.nodes[1].compute = 1. - alpha;
  n.nodes[1].links = {Link{0, D_CONST, 0.0, 0.0}};
  return n;
}

Network Network::selfish_mining(double alpha, double activation_delay, double gamma,
                                double propagation_delay, int defenders) {
  if (defenders < 2) throw std::invalid_argument("defenders must be at least 2");
  double defender_compute = (1. - alpha) / (double)defenders;
  double defenders_ = (double)defenders;
  if (gamma > (defenders_ - 1.) / defenders_)
    throw std::invalid_argument("gamma must not be greater ( (defenders - 1) / defenders )");
  double d = (defenders_ - 1.) / defenders_ * propagation_delay / gamma;
  Network n;
  n.flooding = false;
  n.activation_delay = activation_delay;
  int nn = defenders + 1;
  n.nodes.resize(nn);
  for (int i = 0; i < nn; i++) {
    n.nodes[i].compute = i == 0 ? alpha : defender_compute;
    for (int dest = 0; dest < nn; dest++) {
      if (dest == i) continue;
      if (i == 0)
        n.nodes[i].links.push_back(Link{dest, D_UNIFORM, 0.0, d});
      else if (dest == 0)
        n.nodes[i].links.push_back(Link{dest, D_CONST, 0.0, 0.0});
      else
        n.nodes[i].links.push_back(Link{dest, D_CONST, propagation_delay, 0.0});
    }
  }
  return n;
}

// ---------------------------------------------------------------- RNG adapters

OcamlSimRng::OcamlSimRng(OcamlRandom* r_, const Network& net) : r(r_) {
  ev = net.activation_delay;
  // distributions.ml:45-88 (Vose alias table)
  int n = (int)net.nodes.size();
  double sum = 0.0;
  for (auto& x : net.nodes) {
    if (x.compute < 0.) throw std::invalid_argument("negative probability");
    sum += x.compute;
  }
  p.assign(n, 0.0);
  alias.assign(n, -1);
  double scale = (double)n / sum;
  std::vector<std::pair<double, int>> small, large;  // back = list head
  for (int i = 0; i < n; i++) {
    double pi = net.nodes[i].compute * scale;
    if (pi < 1.)
      small.push_back({pi, i});
    else
      large.push_back({pi, i});
  }
  for (;;) {
    if (!small.empty() && !large.empty()) {
      auto s = small.back();
      small.pop_back();
      auto l = large.back();
      large.pop_back();
      p[s.second] = s.first;
      alias[s.second] = l.second;
      double pp = s.first + l.first - 1.;
      if (pp < 1.)
        small.push_back({pp, l.second});
      else
        large.push_back({pp, l.second});
    } else if (!small.empty()) {
      auto s = small.back();
      small.pop_back();
      p[s.second] = 1.;
      alias[s.second] = -1;
    } else if (!large.empty()) {
      auto l = large.back();
      large.pop_back();
      p[l.second] = 1.;
      alias[l.second] = -1;
    } else
      break;
  }
}

int OcamlSimRng::miner(int) {
  int i = r->int_((int)p.size());
  if (alias[i] < 0) return i;
  return r->float_(1.) > p[i] ? alias[i] : i;
}

double OcamlSimRng::act_delay(int) {
  double x = -1. * ev * std::log(r->float_(1.));
  if (!(x > 0.)) throw std::runtime_error("assert failure: exponential x > 0");
  return x;
}

int32_t OcamlSimRng::pow_bits(int) { return r->bits(); }

double OcamlSimRng::link_delay(const Link& l, const Block*) {
  switch (l.kind) {
    case D_CONST: return l.a;
    case D_UNIFORM: return r->float_(l.b - l.a) + l.a;
    case D_EXP: {
      double x = -1. * l.a * std::log(r->float_(1.));
      if (!(x > 0.)) throw std::runtime_error("assert failure: exponential x > 0");
      return x;
    }
  }
  return 0.0;
}

KeyedSimRng::KeyedSimRng(uint64_t seed, uint64_t episode, const Network& net,
                         bool general_weights)
    : ks(seed, episode) {
  ev = net.activation_delay;
  d = (int)net.nodes.size() - 1;
  t_att = alpha_threshold(net.nodes[0].compute);
  if (general_weights) {
    std::vector<double> w;
    for (const NetNode& x : net.nodes) w.push_back(x.compute);
    thr = weight_thresholds(w);
    return;
  }
  for (int i = 2; i < (int)net.nodes.size(); i++)
    if (net.nodes[i].compute != net.nodes[1].compute)
      throw std::invalid_argument("keyed stream needs equal-weight defenders");
}

int KeyedSimRng::miner(int k) {
  if (!thr.empty()) return ks.miner_w((uint32_t)k, thr);
  return ks.miner((uint32_t)k, t_att, d);
}

double KeyedSimRng::act_delay(int j) {
  double x = -1. * ev * cpr_log(ks.act_u((uint32_t)j));
  return x;
}

int32_t KeyedSimRng::pow_bits(int serial) { return (int32_t)ks.pow_bits((uint32_t)serial); }

double KeyedSimRng::link_delay(const Link& l, const Block* m) {
  const uint32_t kw = (uint32_t)m->share_k, off = (uint32_t)m->share_off;
  if (serial_links) {
    const double u = ks.msg_u((uint32_t)m->serial, (uint32_t)l.dest);
    switch (l.kind) {
      case D_CONST: return l.a;
      case D_UNIFORM: return u * (l.b - l.a) + l.a;
      case D_EXP: return -1. * l.a * cpr_log(u);
    }
  }
  switch (l.kind) {
    case D_CONST: return l.a;
    case D_UNIFORM: return ks.link_u(kw, off, (uint32_t)l.dest) * (l.b - l.a) + l.a;
    case D_EXP: return -1. * l.a * cpr_log(ks.link_u(kw, off, (uint32_t)l.dest));
  }
  return 0.0;
}

// ---------------------------------------------------------------- traces

thread_local TraceHook g_trace;

uint64_t trace_link_key(uint32_t kw, uint32_t off, uint32_t dest) {
  return ((uint64_t)kw << 32) | ((uint64_t)(off & 0xFFFFFu) << 12) | (uint64_t)(dest & 0xFFFu);
}
uint64_t trace_msg_key(uint32_t serial, uint32_t dest) {
  return ((uint64_t)serial << 32) | (uint64_t)(dest & 0xFFFu);
}

namespace {

template <class T>
void put(std::vector<T>& v, int i, T x, T fill) {
  if ((int)v.size() <= i) v.resize(i + 1, fill);
  v[i] = x;
}

uint64_t msg_key_of(const Link& l, const Block* m, bool serial_links) {
  return serial_links ? trace_msg_key((uint32_t)m->serial, (uint32_t)l.dest)
                      : trace_link_key((uint32_t)m->share_k, (uint32_t)m->share_off,
                                       (uint32_t)l.dest);
}

// every draw of `inner`, logged by coordinate (a re-draw at the same coordinate, as when
// the gym's reset runs Simulator.init twice, overwrites)
struct RecordingSimRng : SimRng {
  std::unique_ptr<SimRng> inner;
  TraceBuf* buf;
  bool serial_links;
  int miner(int k) override {
    const int m = inner->miner(k);
    put<int32_t>(buf->miner, k, m, 0);
    return m;
  }
  double act_delay(int j) override {
    const double x = inner->act_delay(j);
    put<double>(buf->delay, j, x, 0.0);
    return x;
  }
  int32_t pow_bits(int serial) override {
    const int32_t p = inner->pow_bits(serial);
    put<int32_t>(buf->pow, serial, p, 0);
    return p;
  }
  double link_delay(const Link& l, const Block* m) override {
    const double x = inner->link_delay(l, m);
    if (l.kind != D_CONST) buf->link[msg_key_of(l, m, serial_links)] = x;
    return x;
  }
  double coin(int kw, int j) override { return inner->coin(kw, j); }
  int rand_action(int i, int n) override { return inner->rand_action(i, n); }
};

struct ReplaySimRng : SimRng {
  TraceBuf* buf;
  bool serial_links;
  int miner(int k) override {
    if (k < (int)buf->miner.size()) return buf->miner[k];
    buf->miss = 1;
    return 0;
  }
  double act_delay(int j) override {
    if (j < (int)buf->delay.size()) return buf->delay[j];
    buf->miss = 1;
    return 1.0;
  }
  int32_t pow_bits(int serial) override {
    if (serial < (int)buf->pow.size()) return buf->pow[serial];
    buf->miss = 1;
    return 0;
  }
  double link_delay(const Link& l, const Block* m) override {
    if (l.kind == D_CONST) return l.a;
    auto it = buf->link.find(msg_key_of(l, m, serial_links));
    if (it != buf->link.end()) return it->second;
    buf->miss = 1;
    return 0.0;
  }
  int rand_action(int, int) override {  // traces hold no policy draws
    buf->miss = 1;
    return 0;
  }
};

}  // namespace

std::unique_ptr<SimRng> trace_wrap(std::unique_ptr<SimRng> inner, const Network& net,
                                   bool serial_links) {
  if (g_trace.mode == TRACE_RECORD) {
    auto* r = new RecordingSimRng();
    r->inner = g_trace.ocaml ? std::unique_ptr<SimRng>(new OcamlSimRng(g_trace.ocaml, net))
                             : std::move(inner);
    r->buf = g_trace.buf;
    r->serial_links = serial_links;
    return std::unique_ptr<SimRng>(r);
  }
  if (g_trace.mode == TRACE_REPLAY) {
    auto* r = new ReplaySimRng();
    r->buf = g_trace.buf;
    r->serial_links = serial_links;
    return std::unique_ptr<SimRng>(r);
  }
  return inner;
}

// ---------------------------------------------------------------- Simulator

Sim::Sim(const Network& net_, SimRng* rng_) : net(net_), rng(rng_) {
  n_nodes = (int)net.nodes.size();
}

// simulator.ml:233-332
void Sim::init(std::vector<std::unique_ptr<NodeImpl>> nodes_) {
  // roots: Protocol.roots = [ {height=0; miner=None} ]
  auto r = std::make_unique<Block>();
  r->serial = 0;
  r->depth = 1;  // dag.ml:29  fold max 0 [] + 1
  r->value = NakData{0, -1};
  r->vis.assign(n_nodes, Vis{RECEIVED, 0.0});
  r->received_at.assign(n_nodes, 0.0);
  r->rewards.assign(n_nodes, 0.0);
  roots.insert(roots.begin(), r.get());
  dag.push_back(std::move(r));
  nodes = std::move(nodes_);
  for (int i = 0; i < n_nodes; i++) {
    nodes[i]->sim = this;
    nodes[i]->id = i;
  }
  activations.assign(n_nodes, 0);
  schedule_pow();
}

void Sim::schedule(double delay, const Event& ev) {
  int id = (int)events.size();
  events.push_back(ev);
  double t = now + delay;
  if (ev.type == EV_NET_RX && std::isfinite(t)) pending_finite_rx++;
  queue.queue(t, id);
}

// simulator.ml:170-173
void Sim::schedule_pow() {
  double x = rng->act_delay(c_activations);
  schedule(x, Event{EV_CLOCK, 0, K_POW, nullptr, -1});
}

bool Sim::validity(const Block* b) const {
  if (proto == 1) return eth_validity(b);
  if (proto == 2) return bk_validity(b, bk_k);
  if (proto == 3) return ts_validity(b, bk_k);
  if (!b->has_pow || b->parents.size() != 1) return false;
  return b->value.height == b->parents[0]->value.height + 1 && b->value.miner >= 0;
}

void Sim::reward(Block* x) const {
  if (proto == 1) {
    eth_reward(x, eth_scheme, x->rewards);
    return;
  }
  if (proto == 2) {
    bk_reward(x, bk_scheme, bk_k, x->rewards);
    return;
  }
  if (proto == 3) {
    ts_reward(x, bk_scheme, bk_k, x->rewards);
    return;
  }
  if (x->value.miner >= 0) x->rewards[x->value.miner] += 1.;
}

// simulator.ml:122-136
Block* Sim::raw_append(bool pow, int node, const Draft& d) {
  if (zt_limit > 0 && ++zt_appends > zt_limit)
    throw std::runtime_error("zero-time append loop: more appends between two activations than the guard allows");
  auto v = std::make_unique<Block>();
  v->serial = (int)dag.size();
  if (pow) {
    v->has_pow = true;
    v->pow_hash = rng->pow_bits(v->serial);
  }
  v->signature = d.sign ? node : -1;
  v->vis.assign(n_nodes, Vis{});
  v->received_at.assign(n_nodes, 1.0 / 0.0);
  v->rewards.assign(n_nodes, std::nan(""));
  v->value = d.data;
  v->parents = d.parents;
  int depth = 0;
  for (auto* p : d.parents) depth = std::max(depth, p->depth);
  v->depth = depth + 1;
  Block* raw = v.get();
  if (d.parents.empty()) roots.insert(roots.begin(), raw);
  for (auto* p : d.parents) p->children_app.push_back(raw);
  dag.push_back(std::move(v));
  return raw;
}

// simulator.ml:139-159 and 390-399
Block* Sim::append(bool pow, int node, const Draft& d) {
  if (!(pow || d.sign)) {
    std::vector<Block*> candidates;
    if (d.parents.empty())
      candidates = roots;
    else
      candidates.assign(d.parents[0]->children_app.rbegin(), d.parents[0]->children_app.rend());
    for (auto* y : candidates) {
      if (!(y->value == d.data) || y->signature != -1) continue;
      // List.for_all2 (stdlib list.ml): false at the first unequal pair; raises
      // Invalid_argument only if all compared pairs are equal and the lengths differ
      bool eq = true;
      size_t i = 0;
      for (; i < y->parents.size() && i < d.parents.size(); i++)
        if (y->parents[i]->serial != d.parents[i]->serial) {
          eq = false;
          break;
        }
      if (eq && y->parents.size() != d.parents.size())
        throw std::invalid_argument("List.for_all2");
      if (eq) return y;  // `Redundant
    }
  }
  Block* x = raw_append(pow, node, d);
  if (!validity(x)) throw std::runtime_error("invalid append");
  // set_rewards: precursor = first parent (nakamoto.ml:50)
  Block* pre = x->parents.empty() ? nullptr : x->parents[0];
  if (!pre) throw std::runtime_error("Referee.precursor should go back to DAG root.");
  x->rewards = pre->rewards;
  reward(x);
  return x;
}

// simulator.ml:401-419
void Sim::handle_action(int node, const Action& act) {
  struct Rec {
    Sim* s;
    int node;
    int off;
    void share(Block* msg) {
      Vis& v = msg->vis[node];
      switch (v.kind) {
        case INVISIBLE: throw std::runtime_error("invalid share");
        case RECEIVED:
        case RELEASED: return;
        case WITHHELD:
          s->schedule_now(Event{EV_NET_TX, node, K_NETWORK, msg, -1});
          v.kind = RELEASED;
          msg->share_k = s->c_activations;
          msg->share_off = off++;
          for (auto* p : msg->parents) share(p);
          return;
      }
    }
  } rec{this, node, 0};
  for (auto* b : act.share) rec.share(b);
  for (auto& d : act.append) {
    int id = (int)drafts.size();
    drafts.push_back(d);
    schedule_now(Event{EV_DAG, node, K_APPEND, nullptr, id});
  }
}

// simulator.ml:421-508
void Sim::handle_event(const Event& ev) {
  switch (ev.type) {
    case EV_MAKEVIS: {
      Block* vtx = ev.blk;
      int n = ev.node;
      bool ok = !visible(n, vtx);
      if (ok)
        for (auto* p : vtx->parents)
          if (!visible(n, p)) ok = false;
      if (ok) {
        vtx->vis[n] = Vis{ev.kind == K_NETWORK ? RECEIVED : WITHHELD, now};
        schedule_now(Event{EV_ONNODE, n, ev.kind, vtx, -1});
        schedule_now(Event{EV_MADEVIS, n, ev.kind, vtx, -1});
      }
      break;
    }
    case EV_ONNODE: {
      int n = ev.node;
      if (!visible(n, ev.blk)) throw std::runtime_error("assert: OnNode invisible");
      for (auto* p : ev.blk->parents)
        if (!visible(n, p)) throw std::runtime_error("assert: OnNode parent invisible");
      if (ev.kind == K_NETWORK && n != 0 && proto < 2) {
        // diagnostic: equal-height candidate delivered at the same instant as the current tip
        Block* cur = nodes[n]->preferred();
        if (cur && cur != ev.blk && cur->value.height == ev.blk->value.height &&
            cur->vis[n].time == now && cur->serial != 0)
          diag |= DIAG_TIE;
      }
      Action act = nodes[n]->handler(ev.kind, ev.blk);
      handle_action(n, act);
      break;
    }
    case EV_CLOCK: {
      if (pending_finite_rx > 0) diag |= DIAG_OVERLAP;
      zt_appends = 0;
      int node_id = rng->miner(c_activations);
      Draft d = nodes[node_id]->puzzle_payload();
      int id = (int)drafts.size();
      drafts.push_back(d);
      schedule_now(Event{EV_DAG, node_id, K_POW, nullptr, id});
      c_activations++;
      activations[node_id]++;
      schedule_pow();
      break;
    }
    case EV_DAG: {
      bool pow = ev.kind == K_POW;
      Block* v = append(pow, ev.node, drafts[ev.draft]);
      schedule_now(Event{EV_MAKEVIS, ev.node, pow ? K_POW : K_APPEND, v, -1});
      break;
    }
    case EV_NET_TX: {
      for (auto& l : net.nodes[ev.node].links) {
        double delay = rng->link_delay(l, ev.blk);
        schedule(delay, Event{EV_NET_RX, l.dest, K_NETWORK, ev.blk, -1});
      }
      break;
    }
    case EV_NET_RX: {
      int n = ev.node;
      if (now < ev.blk->received_at[n]) {
        ev.blk->received_at[n] = now;
        schedule_now(Event{EV_MAKEVIS, n, K_NETWORK, ev.blk, -1});
      }
      break;
    }
    case EV_MADEVIS: {
      int n = ev.node;
      Block* vtx = ev.blk;
      if (net.flooding && vtx->received_at[n] <= now)
        schedule_now(Event{EV_NET_TX, n, K_NETWORK, vtx, -1});
      for (auto it = vtx->children_app.rbegin(); it != vtx->children_app.rend(); ++it) {
        Block* c = *it;
        if (c->received_at[n] <= now) schedule_now(Event{EV_MAKEVIS, n, K_NETWORK, c, -1});
      }
      break;
    }
  }
}

// simulator.ml:510-517
bool Sim::dequeue(Event* ev) {
  double t;
  int id;
  if (!queue.dequeue(&t, &id)) return false;
  if (!(t >= now)) throw std::runtime_error("assert: now >= clock.now");
  now = t;
  *ev = events[id];
  if (ev->type == EV_NET_RX && std::isfinite(t)) pending_finite_rx--;
  return true;
}

// simulator.ml:519-533
void Sim::loop(int acts) {
  Event ev;
  int left = acts;
  while (dequeue(&ev)) {
    if (ev.type == EV_CLOCK) {
      if (left <= 0) continue;
      handle_event(ev);
      left--;
    } else
      handle_event(ev);
  }
}

// nakamoto.ml:43-48
Block* Sim::winner(const std::vector<Block*>& l) {
  if (l.empty()) throw std::runtime_error("nakamoto.winner: empty list");
  Block* acc = l[0];
  for (size_t i = 1; i < l.size(); i++)
    if (l[i]->value.height > acc->value.height) acc = l[i];
  return acc;
}

// simulator.ml:535-543
Block* Sim::head() {
  std::vector<Block*> prefs;
  for (auto& n : nodes) prefs.push_back(n->preferred());
  return winner(prefs);
}

// simulator.ml:14-21
double Sim::timestamp(const Block* b) {
  double m = 1.0 / 0.0;
  for (auto& v : b->vis) {
    double x = v.kind == INVISIBLE ? 1.0 / 0.0 : v.time;
    m = std::fmin(m, x);
  }
  return m;
}

// dagtools.ml:73-121: ordered ancestor iteration by (depth, serial), merged
Block* common_ancestor(const Sim& sim, int view, Block* a, Block* b) {
  auto key = [](Block* x) { return std::make_pair(x->depth, x->serial); };
  struct Cmp {
    bool operator()(Block* x, Block* y) const {
      if (x->depth != y->depth) return x->depth > y->depth;
      return x->serial > y->serial;
    }
  };
  std::set<Block*, Cmp> qa{a}, qb{b};
  auto next = [&](std::set<Block*, Cmp>& q) -> Block* {
    if (q.empty()) return nullptr;
    Block* v = *q.begin();
    q.erase(q.begin());
    for (auto* p : v->parents)
      if (sim.visible(view, p)) q.insert(p);
    return v;
  };
  Block* x = next(qa);
  Block* y = next(qb);
  while (x && y) {
    auto kx = key(x), ky = key(y);
    if (kx == ky) return x;
    if (kx > ky)
      x = next(qa);
    else
      y = next(qb);
  }
  return nullptr;
}

// ---------------------------------------------------------------- Nakamoto honest

Draft NakHonest::puzzle_payload() {
  Draft d;
  d.parents = {state};
  d.data = NakData{state->value.height + 1, id};
  d.sign = false;
  return d;
}

// nakamoto.ml:85-95
Action NakHonest::handler(Kind k, Block* v) {
  Action a;
  switch (k) {
    case K_APPEND: throw std::runtime_error("not implemented");
    case K_NETWORK:
      if (v->value.height > state->value.height) {
        state = v;
      } else if (abstract_gamma >= 0.0 && v != state && v->value.height == state->value.height) {
        // abstract-gamma match race: the attacker's release against the defender block
        // mined at this very instant, in either arrival order; the coin decides
        Block* att = v->value.miner == 0 ? v : (state->value.miner == 0 ? state : nullptr);
        Block* def = att == v ? state : v;
        if (att && def->value.miner >= 1 && def->vis[def->value.miner].time == sim->now)
          state = sim->rng->coin(att->share_k, id) < abstract_gamma ? att : def;
      }
      return a;
    case K_POW:
      state = v;
      a.share = {v};
      return a;
  }
  return a;
}

Draft DummyNode::puzzle_payload() {
  Draft d;
  d.parents = {state};
  d.data = NakData{state->value.height + 1, id};
  return d;
}
Action DummyNode::handler(Kind, Block*) {
  throw std::runtime_error("dummy node handler must not be called");
}

// ---------------------------------------------------------------- SSZ attack space

// nakamoto_ssz.ml:274-340
int nak_policy(int policy, const NakObs& o, const TablePolicy* table) {
  const int h = o.public_blocks, a = o.private_blocks;
  switch (policy) {
    case POL_HONEST:
      if (a > h) return OVERRIDE;
      if (a < h) return ADOPT;
      return WAIT;
    case POL_SIMPLE:
      if (h > 0) return a < h ? ADOPT : OVERRIDE;
      return WAIT;
    case POL_ES2014:
      if (a < h) return ADOPT;
      if (h == 0 && a == 1) return WAIT;
      if (h == 1 && a == 1) return MATCH;
      if (h == 1 && a == 2) return OVERRIDE;
      if (h == 2 && a == 1) return ADOPT;
      if (h > 0) return (a - h == 1) ? OVERRIDE : MATCH;
      return WAIT;
    case POL_SM1:
      if (h > a) return ADOPT;
      if (h == 1 && a == 1) return MATCH;
      if (h == a - 1 && h >= 1) return OVERRIDE;
      return WAIT;
    case POL_TABLE: {
      int dim = table->dim;
      int hp = std::min(std::max(h, 0), dim - 1);
      int ap = std::min(std::max(a, 0), dim - 1);
      return table->actions[(hp * dim + ap) * 2 + o.event];
    }
  }
  throw std::invalid_argument("unknown policy");
}

// ssz_tools.ml:29-40 (unit) and 11-18 (raw); field order nakamoto_ssz.ml:24-30
void nak_obs_to_floats(const NakObs& o, bool unit, double out[4]) {
  if (unit) {
    out[0] = 2. / M_PI * std::atan((double)o.public_blocks / 1.0);
    out[1] = 2. / M_PI * std::atan((double)o.private_blocks / 1.0);
    out[2] = 0.5 + (1. / M_PI * std::atan((double)o.diff_blocks / 1.0));
    out[3] = (double)o.event / 1.0;
  } else {
    out[0] = (double)o.public_blocks;
    out[1] = (double)o.private_blocks;
    out[2] = (double)o.diff_blocks;
    out[3] = (double)o.event;
  }
}

static long ocaml_round_to_int(double x) { return (long)std::round(x); }

// ssz_tools.ml:11-59
NakObs nak_obs_of_floats(const double in[4], bool unit) {
  NakObs o;
  if (unit) {
    o.public_blocks = (int)ocaml_round_to_int(std::tan(M_PI / 2. * in[0]) * 1.0);
    o.private_blocks = (int)ocaml_round_to_int(std::tan(M_PI / 2. * in[1]) * 1.0);
    o.diff_blocks = (int)ocaml_round_to_int(std::tan(M_PI * (in[2] - 0.5)) * 1.0);
    o.event = (int)std::floor(in[3] * 1.0);
  } else {
    o.public_blocks = (int)in[0];
    o.private_blocks = (int)in[1];
    o.diff_blocks = (int)in[2];
    o.event = (int)in[3];
  }
  return o;
}

Draft NakSszAgent::puzzle_payload() const {
  Draft d;
  d.parents = {priv};
  d.data = NakData{priv->value.height + 1, my_id};
  return d;
}

// nakamoto_ssz.ml:191-218
void NakSszAgent::prepare(Kind k, Block* x) {
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

// nakamoto_ssz.ml:220-230
NakObs NakSszAgent::observe() const {
  int ca = o_common->value.height, pr = o_priv->value.height, pu = o_pub->value.height;
  return NakObs{pu - ca, pr - ca, pr - pu, o_event};
}

// nakamoto_ssz.ml:232-260
Action NakSszAgent::apply(int action) {
  auto match_ = [&](int offset) {
    int h = o_pub->value.height + offset;
    Block* b = o_priv;
    while (b->value.height > h) {
      std::vector<Block*> vp;
      for (auto* x : b->parents)
        if (sim->visible(my_id, x)) vp.push_back(x);
      if (vp.size() != 1) throw std::runtime_error("Option.get");
      b = vp[0];
    }
    return b;
  };
  Action a;
  Block* np = o_priv;
  switch (action) {
    case ADOPT: np = o_pub; break;
    case MATCH: a.share = {match_(0)}; break;
    case OVERRIDE: a.share = {match_(1)}; break;
    case WAIT: break;
    default: throw std::invalid_argument("Invalid_argument index out of bounds");
  }
  pub = o_pub;
  priv = np;
  pending = a.share;
  return a;
}

Action NakSszAttackerNode::handler(Kind k, Block* b) {
  agent.prepare(k, b);
  int act = policy == POL_RANDOM ? agent.sim->rng->rand_action(nrand++, 4)
                                 : nak_policy(policy, agent.observe(), table);
  return agent.apply(act);
}

// ---------------------------------------------------------------- Gym engine

std::string gym_params_error(const GymParams& p) {
  if (std::isnan(p.activation_delay)) return "activation_delay cannot be NaN";
  if (std::isnan(p.alpha)) return "alpha cannot be NaN";
  if (std::isnan(p.gamma)) return "gamma cannot be NaN";
  if (p.alpha < 0. || p.alpha > 1.) return "alpha < 0 || alpha > 1";
  if (p.gamma < 0. || p.gamma > 1.) return "gamma < 0 || gamma > 1";
  if (p.defenders < 1) return "defenders < 0";
  if (p.activation_delay <= 0.) return "activation_delay <= 0";
  if (p.max_steps <= 0) return "max_steps <= 0";
  if (p.max_progress <= 0.) return "max_progress <= 0";
  if (p.max_time <= 0.) return "max_time <= 0";
  return "";
}

GymNakamoto::GymNakamoto(const GymParams& p_, int mode, OcamlRandom* oc, uint64_t seed_,
                         uint64_t ep)
    : p(p_), rng_mode(mode), ocaml(oc), seed(seed_), episode(ep) {
  std::string e = gym_params_error(p);
  if (!e.empty()) throw std::invalid_argument(e);
  if (p.abstract_gamma) {
    // flagged abstract-gamma mode: the gym's nodes and compute, every link delay zero
    net = Network{};
    net.activation_delay = p.activation_delay;
    net.nodes.resize(p.defenders + 1);
    net.nodes[0].compute = p.alpha;
    for (int i = 1; i <= p.defenders; ++i) net.nodes[i].compute = (1. - p.alpha) / p.defenders;
    for (int i = 0; i <= p.defenders; ++i)
      for (int j = 0; j <= p.defenders; ++j)
        if (j != i) net.nodes[i].links.push_back(Link{j, D_CONST, 0.0, 0.0});
    return;
  }
  // engine.ml:100-107
  net = Network::selfish_mining(p.alpha, p.activation_delay, p.gamma, p.propagation_delay,
                                p.defenders);
}

// engine.ml:108-121
Kind GymNakamoto::skip_to_interaction(Block** blk) {
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

// engine.ml:122-156
void GymNakamoto::init() {
  if (rng_mode == 0)
    rng.reset(new OcamlSimRng(ocaml, net));
  else
    rng.reset(new KeyedSimRng(seed, episode, net));
  rng = trace_wrap(std::move(rng), net, false);
  sim.reset(new Sim(net, rng.get()));
  std::vector<std::unique_ptr<NodeImpl>> nodes;
  int n = (int)net.nodes.size();
  for (int i = 0; i < n; i++) {
    if (i == 0)
      nodes.emplace_back(new DummyNode());
    else
      nodes.emplace_back(new NakHonest());
  }
  Block* root = nullptr;
  {
    // roots exist only after Sim::init; node init needs them
    sim->init(std::move(nodes));
    root = sim->roots.back();
    for (int i = 0; i < n; i++) {
      if (i == 0)
        static_cast<DummyNode*>(sim->nodes[0].get())->state = root;
      else {
        auto* h = static_cast<NakHonest*>(sim->nodes[i].get());
        h->state = root;
        if (p.abstract_gamma) h->abstract_gamma = p.gamma;
      }
    }
  }
  agent = NakSszAgent();
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

void GymNakamoto::observe(double obs[4]) const { nak_obs_to_floats(agent.observe(), p.unit_obs, obs); }

void GymNakamoto::reset(double obs[4]) {
  init();
  observe(obs);
}

// engine.ml:176-249
double GymNakamoto::step(int action, double obs[4], bool* done, StepInfo* info) {
  Action act = agent.apply(action);
  sim->handle_action(0, act);
  episode_steps++;
  Block* b;
  Kind k = skip_to_interaction(&b);
  Block* attacker_pref = agent.priv;  // BetweenActions state, before prepare
  agent.prepare(k, b);
  std::vector<Block*> prefs;
  prefs.push_back(attacker_pref);
  for (int i = 1; i < sim->n_nodes; i++) prefs.push_back(sim->nodes[i]->preferred());
  Block* head = Sim::winner(prefs);
  double progress = (double)head->value.height;
  *done = !(episode_steps < p.max_steps && progress < p.max_progress && sim->now < p.max_time);
  double ra = 0., rd = 0.;
  for (int i = 0; i < sim->n_nodes; i++) {
    if (i == 0)
      ra += head->rewards[i];
    else
      rd += head->rewards[i];
  }
  double chain_time = Sim::timestamp(head);
  double sim_time = sim->now;
  double reward = ra - last_reward_attacker;
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
  }
  last_chain_time = chain_time;
  last_sim_time = sim_time;
  last_reward_attacker = ra;
  last_reward_defender = rd;
  last_progress = progress;
  observe(obs);
  return reward;
}

}  // namespace oracle

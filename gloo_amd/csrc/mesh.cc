// mesh.cc — a schedule's RESULT with mesh data movement (see mesh.h).
//
// 1. Dataflow.  All P ranks' plans (plan.cc, the reference schedules) are
//    executed symbolically.  A buffer position holds a Value: an expression
//    tree over the ranks' original inputs, the element index it is evaluated
//    at (position + delta) and the rank that built its root.  REDUCE makes
//    Node(user, inbox) — `local op incoming`, the operand order of
//    ReductionFunction::call — SEND/COPY move Values.  Buffers are interval
//    maps, so the cost is O(steps x pieces), independent of the element count.
// 2. Jobs.  For allreduce the final trees (identical on every rank) split
//    [0, count) into jobs: (owner = the rank that built the root, range,
//    tree).  For reduce-scatter every rank's output range is its own job.
// 3. Mesh plan.  Each rank sends its raw piece of every job straight to the
//    job's owner (all peers at once: one xGMI link each on an 8-GPU node);
//    the owner evaluates the SAME tree — one pass when it is a chain
//    (FOLD / FOLD_REVERSE) or a balanced tree (FOLD_TREE), pairwise through
//    arena temporaries otherwise — and, for allreduce, sends the result to
//    every rank.  Identical expression trees => identical bits.
#include "gloo_amd/mesh.h"

#include <algorithm>
#include <functional>
#include <map>
#include <stdexcept>
#include <tuple>

#include "gloo_amd.h"

namespace gloo_amd {

namespace {

struct TreeNode {
  int leaf;  // >= 0: rank's input; -1: internal
  int lhs, rhs;
};

class Forest {
 public:
  int leaf(int r) { return intern(r, -1, -1); }
  int node(int a, int b) { return intern(-1, a, b); }
  const TreeNode& at(int i) const { return nodes_[i]; }

 private:
  int intern(int leaf, int a, int b) {
    const auto key = std::make_tuple(leaf, a, b);
    auto it = ids_.find(key);
    if (it != ids_.end()) return it->second;
    nodes_.push_back({leaf, a, b});
    ids_[key] = (int)nodes_.size() - 1;
    return (int)nodes_.size() - 1;
  }
  std::vector<TreeNode> nodes_;
  std::map<std::tuple<int, int, int>, int> ids_;
};

struct Value {
  int tree = -1;      // -1: unknown contents
  int64_t delta = 0;  // element index = position + delta
  int producer = -1;  // rank that built the root
};

struct Piece {
  uint64_t lo, hi;
  Value v;
};

// Interval map over buffer positions.
class Buffer {
 public:
  std::vector<Piece> read(uint64_t lo, uint64_t hi) const {
    std::vector<Piece> out;
    uint64_t at = lo;
    auto it = m_.upper_bound(lo);
    if (it != m_.begin()) --it;
    for (; at < hi; ) {
      while (it != m_.end() && it->second.hi <= at) ++it;
      if (it == m_.end() || it->second.lo >= hi) {
        out.push_back({at, hi, Value{}});
        break;
      }
      const Piece& p = it->second;
      if (p.lo > at) {
        out.push_back({at, p.lo, Value{}});
        at = p.lo;
      }
      const uint64_t e = std::min(p.hi, hi);
      out.push_back({at, e, p.v});
      at = e;
    }
    return out;
  }
  // Store `pieces` (positions as read) shifted so that position `from`
  // lands at `to`.
  void write(const std::vector<Piece>& pieces, uint64_t from, uint64_t to) {
    if (pieces.empty()) return;
    const uint64_t lo = to, hi = to + (pieces.back().hi - from);
    split(lo);
    split(hi);
    m_.erase(m_.lower_bound(lo), m_.lower_bound(hi));
    for (Piece p : pieces) {
      const int64_t shift = (int64_t)to - (int64_t)from;
      p.lo += shift;
      p.hi += shift;
      p.v.delta -= shift;
      if (p.lo < p.hi) m_[p.lo] = p;
    }
  }

 private:
  void split(uint64_t at) {
    auto it = m_.upper_bound(at);
    if (it == m_.begin()) return;
    --it;
    Piece& p = it->second;
    if (p.lo < at && at < p.hi) {
      Piece q = p;
      q.lo = at;
      p.hi = at;
      m_[at] = q;
    }
  }
  std::map<uint64_t, Piece> m_;
};

struct Job {
  int owner;
  uint64_t lo, hi;  // positions in the owner's user buffer (output)
  uint64_t elem;    // element index of position lo (= lo for allreduce)
  int tree;
};

bool isAllreduce(int algo) {
  return algo == GLOO_HIP_ALGO_RING_CHUNKED || algo == GLOO_HIP_ALGO_HALVING_DOUBLING || algo == GLOO_HIP_ALGO_RING ||
         algo == GLOO_HIP_ALGO_ALLREDUCE_RING || algo == GLOO_HIP_ALGO_ALLREDUCE_BCUBE ||
         algo == GLOO_HIP_ALGO_BCUBE;
}

// Combine aligned piece lists of several operands position by position.
template <typename F>
void zipPieces(const std::vector<std::vector<Piece>>& ops, const std::vector<uint64_t>& offs, uint64_t len, F&& emit) {
  std::vector<size_t> idx(ops.size(), 0);
  for (uint64_t t = 0; t < len;) {
    uint64_t e = len;
    std::vector<const Value*> vs;
    for (size_t k = 0; k < ops.size(); k++) {
      while (ops[k][idx[k]].hi <= offs[k] + t) idx[k]++;
      e = std::min(e, ops[k][idx[k]].hi - offs[k]);
      vs.push_back(&ops[k][idx[k]].v);
    }
    emit(t, e, vs);
    t = e;
  }
}

// Run every rank's plan symbolically; returns the final user buffers.
// New-style algorithms are modelled with one output and no separate input:
// a rank's leaf is its contribution (the local reduction of its inputs,
// which the reference computes range by range before using it).
std::vector<Buffer> dataflow(int algo, int size, uint64_t count, const std::vector<int>& recvElems, Forest& F,
                             const NewStyleOptions* ns) {
  std::vector<Plan> plans;
  NewStyleOptions model;
  if (ns) {
    model = *ns;
    model.ninputs = 0;
    model.noutputs = 1;
  }
  for (int r = 0; r < size; r++)
    plans.push_back(ns ? makeNewStylePlan(algo, r, size, count, model) : makePlan(algo, r, size, count, 1, recvElems));
  std::vector<std::pair<bool, uint64_t>> foldSrcs;  // pending FOLD sources: (arena?, offset)
  std::vector<Buffer> user(size), arena(size);
  for (int r = 0; r < size; r++) {
    std::vector<Piece> init{{0, count, Value{F.leaf(r), 0, r}}};
    if (count) user[r].write(init, 0, 0);
  }
  std::map<std::tuple<int, int, int>, uint64_t> region;  // (src, dst, slot) -> dst arena offset
  for (int r = 0; r < size; r++)
    for (const Step& s : plans[r].steps)
      if (s.kind == GLOO_HIP_STEP_DECL_RECV) region[std::make_tuple(s.peer, r, s.slot)] = s.dst_off;
  std::map<std::tuple<int, int, int>, uint64_t> sent, consumed;
  std::vector<size_t> pc(size, 0);
  auto space = [&](int r, bool isArena) -> Buffer& { return isArena ? arena[r] : user[r]; };
  for (;;) {
    bool progress = false, done = true;
    for (int r = 0; r < size; r++) {
      const auto& steps = plans[r].steps;
      while (pc[r] < steps.size()) {
        const Step& s = steps[pc[r]];
        if (s.kind == GLOO_HIP_STEP_WAIT_RECV || s.kind == GLOO_HIP_STEP_WAIT_NOTIFY) {
          const auto key = std::make_tuple(s.peer, r, s.slot);
          if (sent[key] <= consumed[key]) break;
          consumed[key]++;
        } else if (s.kind == GLOO_HIP_STEP_SEND) {
          const auto key = std::make_tuple(r, s.peer, s.slot);
          auto it = region.find(key);
          if (it == region.end()) throw std::runtime_error("send to an undeclared region");
          const auto pieces = space(r, s.flags & GLOO_HIP_SRC_ARENA).read(s.src_off, s.src_off + s.length);
          arena[s.peer].write(pieces, s.src_off, it->second + s.dst_off);
          sent[key]++;
        } else if (s.kind == GLOO_HIP_STEP_NOTIFY) {
          sent[std::make_tuple(r, s.peer, s.slot)]++;
        } else if (s.kind == GLOO_HIP_STEP_REDUCE) {
          const auto a = user[r].read(s.dst_off, s.dst_off + s.length);
          const auto b = arena[r].read(s.src_off, s.src_off + s.length);
          std::vector<Piece> out;
          size_t ia = 0, ib = 0;
          for (uint64_t t = 0; t < s.length;) {
            while (a[ia].hi <= s.dst_off + t) ia++;
            while (b[ib].hi <= s.src_off + t) ib++;
            const uint64_t e = std::min(a[ia].hi - s.dst_off, b[ib].hi - s.src_off);
            Value v;
            const Value &va = a[ia].v, &vb = b[ib].v;
            if (va.tree >= 0 && vb.tree >= 0) {
              if ((int64_t)(s.dst_off + t) + va.delta != (int64_t)(s.src_off + t) + vb.delta)
                throw std::runtime_error("reduction of different elements");
              v = Value{F.node(va.tree, vb.tree), va.delta, r};
            }
            out.push_back({s.dst_off + t, s.dst_off + e, v});
            t = e;
          }
          user[r].write(out, s.dst_off, s.dst_off);
        } else if (s.kind == GLOO_HIP_STEP_FOLD_SRC) {
          foldSrcs.push_back({(s.flags & GLOO_HIP_SRC_ARENA) != 0, s.src_off});
        } else if (s.kind == GLOO_HIP_STEP_FOLD) {
          // acc = s0; acc = acc op s_k (REVERSE: s_k op acc; TREE: pairwise)
          std::vector<std::vector<Piece>> ops;
          std::vector<uint64_t> offs;
          for (const auto& fs : foldSrcs) {
            ops.push_back(space(r, fs.first).read(fs.second, fs.second + s.length));
            offs.push_back(fs.second);
          }
          foldSrcs.clear();
          std::vector<Piece> out;
          zipPieces(ops, offs, s.length, [&](uint64_t t, uint64_t e, const std::vector<const Value*>& vs) {
            bool known = true;
            for (size_t k = 0; k < vs.size(); k++) {
              if (vs[k]->tree < 0) known = false;
              else if ((int64_t)(offs[k] + t) + vs[k]->delta != (int64_t)(offs[0] + t) + vs[0]->delta)
                throw std::runtime_error("fold of different elements");
            }
            Value v;
            if (known) {
              std::vector<int> level;
              for (const Value* x : vs) level.push_back(x->tree);
              int acc;
              if (s.flags & GLOO_HIP_FOLD_TREE) {
                while (level.size() > 1) {
                  std::vector<int> next;
                  for (size_t k = 0; k + 1 < level.size(); k += 2) next.push_back(F.node(level[k], level[k + 1]));
                  level = next;
                }
                acc = level[0];
              } else {
                acc = level[0];
                for (size_t k = 1; k < level.size(); k++)
                  acc = s.flags & GLOO_HIP_FOLD_REVERSE ? F.node(level[k], acc) : F.node(acc, level[k]);
              }
              // element index as seen from the destination position
              v = Value{acc, (int64_t)(offs[0] + t) + vs[0]->delta - (int64_t)(s.dst_off + t), r};
            }
            out.push_back({s.dst_off + t, s.dst_off + e, v});
          });
          space(r, s.flags & GLOO_HIP_DST_ARENA).write(out, s.dst_off, s.dst_off);
        } else if (s.kind == GLOO_HIP_STEP_COPY) {
          const auto pieces = space(r, s.flags & GLOO_HIP_SRC_ARENA).read(s.src_off, s.src_off + s.length);
          space(r, s.flags & GLOO_HIP_DST_ARENA).write(pieces, s.src_off, s.dst_off);
        } else if (s.kind == GLOO_HIP_STEP_DECL_RECV || s.kind == GLOO_HIP_STEP_WAIT_SEND) {
        } else {
          throw std::runtime_error("step kind outside the dataflow model");
        }
        pc[r]++;
        progress = true;
      }
      if (pc[r] < steps.size()) done = false;
    }
    if (done) break;
    if (!progress) throw std::runtime_error("schedule deadlocks");
  }
  return user;
}

int countLeaves(const Forest& F, int t) {
  const TreeNode& n = F.at(t);
  return n.leaf >= 0 ? 1 : countLeaves(F, n.lhs) + countLeaves(F, n.rhs);
}

std::vector<Job> findJobs(int algo, int size, uint64_t count, const std::vector<int>& recvElems, Forest& F,
                          const NewStyleOptions* ns) {
  const auto user = dataflow(algo, size, count, recvElems, F, ns);
  std::vector<Job> jobs;
  auto add = [&](int owner, const Piece& p) {
    if (p.v.tree < 0) throw std::runtime_error("output element with unknown contents");
    if (countLeaves(F, p.v.tree) != size) throw std::runtime_error("output is not a full reduction");
    const uint64_t elem = (uint64_t)((int64_t)p.lo + p.v.delta);
    if (!jobs.empty()) {
      Job& b = jobs.back();
      if (b.owner == owner && b.tree == p.v.tree && b.hi == p.lo && b.elem + (b.hi - b.lo) == elem) {
        b.hi = p.hi;
        return;
      }
    }
    jobs.push_back({owner, p.lo, p.hi, elem, p.v.tree});
  };
  if (isAllreduce(algo)) {
    const auto ref = user[0].read(0, count);
    for (int r = 1; r < size; r++) {
      const auto other = user[r].read(0, count);
      size_t i = 0, j = 0;
      for (uint64_t t = 0; t < count;) {
        while (ref[i].hi <= t) i++;
        while (other[j].hi <= t) j++;
        if (ref[i].v.tree != other[j].v.tree || ref[i].v.delta != other[j].v.delta)
          throw std::runtime_error("ranks end with different results");
        t = std::min(ref[i].hi, other[j].hi);
      }
    }
    for (const Piece& p : ref) {
      if (p.v.delta != 0) throw std::runtime_error("allreduce output misplaced");
      add(p.v.producer, p);
    }
  } else if (algo == GLOO_HIP_ALGO_REDUCE_SCATTER) {
    for (int r = 0; r < size; r++)
      for (const Piece& p : user[r].read(0, (uint64_t)recvElems[r])) add(r, p);
  } else if (algo == GLOO_HIP_ALGO_REDUCE && ns) {
    // gloo::reduce: the root's output; each range is owned by the rank that
    // finished its tree (the reference then gathers it at the root)
    for (const Piece& p : user[ns->root].read(0, count)) {
      if (p.v.delta != 0) throw std::runtime_error("reduce output misplaced");
      add(p.v.producer, p);
    }
  } else {
    throw std::runtime_error("no mesh form for this algorithm");
  }
  return jobs;
}

// Leaf order of a chain / balanced tree, or empty when the shape is neither.
bool rightChain(const Forest& F, int t, std::vector<int>& order) {  // s_k op (... (s_1 op s_0))
  const TreeNode& n = F.at(t);
  if (n.leaf >= 0) {
    order.push_back(n.leaf);
    return true;
  }
  if (F.at(n.lhs).leaf < 0) return false;
  if (!rightChain(F, n.rhs, order)) return false;
  order.push_back(F.at(n.lhs).leaf);
  return true;
}
bool leftChain(const Forest& F, int t, std::vector<int>& order) {  // ((s_0 op s_1) op s_2) ...
  const TreeNode& n = F.at(t);
  if (n.leaf >= 0) {
    order.push_back(n.leaf);
    return true;
  }
  if (F.at(n.rhs).leaf < 0) return false;
  if (!leftChain(F, n.lhs, order)) return false;
  order.push_back(F.at(n.rhs).leaf);
  return true;
}
int balanced(const Forest& F, int t, std::vector<int>& order) {  // depth, or -1
  const TreeNode& n = F.at(t);
  if (n.leaf >= 0) {
    order.push_back(n.leaf);
    return 0;
  }
  const int a = balanced(F, n.lhs, order);
  const int b = balanced(F, n.rhs, order);
  return (a < 0 || a != b) ? -1 : a + 1;
}

Step mkStep(int kind, int peer = -1, int slot = 0, int flags = 0, uint64_t dst = 0, uint64_t src = 0,
            uint64_t len = 0) {
  Step s;
  s.kind = kind;
  s.peer = peer;
  s.slot = slot;
  s.flags = flags;
  s.dst_off = dst;
  s.src_off = src;
  s.length = len;
  return s;
}

}  // namespace

Plan makeMeshPlan(int algo, int rank, int size, uint64_t count, int nptrs, const std::vector<int>& recvElems,
                  const NewStyleOptions* ns) {
  if (size < 2 || size > GLOO_HIP_MAX_SRCS) throw std::invalid_argument("mesh plans need 2 <= size <= 8");
  if (rank < 0 || rank >= size) throw std::invalid_argument("bad rank");
  Plan p;
  const bool allreduce = isAllreduce(algo);
  const bool toRoot = algo == GLOO_HIP_ALGO_REDUCE;  // gloo::reduce: results go to the root only
  if (toRoot && !ns) throw std::invalid_argument("gloo::reduce needs its options");
  if (count == 0) return p;
  // A rank's contribution: the local reduction of its inputs (new-style,
  // the reference's reduceInputs over the whole range), or of its pointers.
  // gloo::reduce reads its single input in place (leafFlags).
  const int leafFlags = toRoot && ns->ninputs > 0 ? GLOO_HIP_FROM_INPUTS : 0;
  if (ns && !toRoot && ns->ninputs > 0)
    p.steps.push_back(mkStep(GLOO_HIP_STEP_LOCAL_REDUCE, -1, 0, GLOO_HIP_FROM_INPUTS, 0, 0, count));
  else if (nptrs > 1)
    p.steps.push_back(mkStep(GLOO_HIP_STEP_LOCAL_REDUCE, -1, 0, 0, 0, 0, count));
  Forest F;
  const std::vector<Job> jobs = findJobs(algo, size, count, recvElems, F, ns);
  // per owner: its jobs (<= 2: two data slots per direction)
  std::vector<std::vector<int>> byOwner(size);
  for (int j = 0; j < (int)jobs.size(); j++) byOwner[jobs[j].owner].push_back(j);
  for (int o = 0; o < size; o++)
    if (byOwner[o].size() > 2) throw std::runtime_error("more than two output ranges on one rank");
  auto slotOf = [&](int j, int base) {
    const auto& v = byOwner[jobs[j].owner];
    return base + (int)(std::find(v.begin(), v.end(), j) - v.begin());
  };
  uint64_t top = 0;
  auto alloc = [&](uint64_t n) {
    const uint64_t off = top;
    top += std::max<uint64_t>(n, 1);
    return off;
  };
  std::map<std::pair<int, int>, uint64_t> rsRegion;  // (job, sender) -> arena offset
  std::map<int, uint64_t> agRegion;                  // job -> arena offset
  auto peersFrom = [&](int me) {
    std::vector<int> v;
    for (int d = 1; d < size; d++) v.push_back((me + d) % size);
    return v;
  };
  for (int j : byOwner[rank])
    for (int s : peersFrom(rank)) {
      rsRegion[{j, s}] = alloc(jobs[j].hi - jobs[j].lo);
      p.steps.push_back(mkStep(GLOO_HIP_STEP_DECL_RECV, s, slotOf(j, GLOO_HIP_SLOT_DATA0), 0, rsRegion[{j, s}], 0,
                               jobs[j].hi - jobs[j].lo));
    }
  if (allreduce)
    for (int o : peersFrom(rank))
      for (int j : byOwner[o]) {
        agRegion[j] = alloc(jobs[j].hi - jobs[j].lo);
        p.steps.push_back(mkStep(GLOO_HIP_STEP_DECL_RECV, o, slotOf(j, GLOO_HIP_SLOT_AUX0), 0, agRegion[j], 0,
                                 jobs[j].hi - jobs[j].lo));
      }
  std::map<int, uint64_t> rootRegion;  // job -> root's arena offset (gloo::reduce)
  if (toRoot && rank == ns->root)
    for (int o : peersFrom(rank))
      for (int j : byOwner[o]) {
        rootRegion[j] = alloc(jobs[j].hi - jobs[j].lo);
        p.steps.push_back(mkStep(GLOO_HIP_STEP_DECL_RECV, o, slotOf(j, GLOO_HIP_SLOT_AUX0), 0, rootRegion[j], 0,
                                 jobs[j].hi - jobs[j].lo));
      }
  // Reduce-scatter has no return hop, so an owner hands back a credit once
  // its folds have read the inboxes; a sender's next-run send waits for it.
  if (!allreduce)
    for (int o : peersFrom(rank))
      if (!byOwner[o].empty())
        p.steps.push_back(mkStep(GLOO_HIP_STEP_WAIT_NOTIFY, o, GLOO_HIP_SLOT_NOTIFY, GLOO_HIP_PREV_RUN));
  // my raw piece of every other owner's jobs, all at once
  for (int o : peersFrom(rank))
    for (int j : byOwner[o])
      p.steps.push_back(mkStep(GLOO_HIP_STEP_SEND, o, slotOf(j, GLOO_HIP_SLOT_DATA0), leafFlags, 0, jobs[j].elem,
                               jobs[j].hi - jobs[j].lo));
  if (!byOwner[rank].empty()) {
    for (int j : byOwner[rank])
      for (int s : peersFrom(rank)) p.steps.push_back(mkStep(GLOO_HIP_STEP_WAIT_RECV, s, slotOf(j, GLOO_HIP_SLOT_DATA0)));
    for (int j : byOwner[rank]) {
      const Job& J = jobs[j];
      const uint64_t len = J.hi - J.lo;
      // where each leaf lives: peers' inboxes, or my own input in place —
      // staged to the arena if it overlaps the output at another offset
      std::map<int, std::pair<int, uint64_t>> leafAt;  // rank -> (FOLD_SRC flags, offset)
      for (int s : peersFrom(rank)) leafAt[s] = {GLOO_HIP_SRC_ARENA, rsRegion[{j, s}]};
      const bool overlap = J.elem != J.lo && J.elem < J.hi && J.lo < J.elem + len;
      if (overlap) {
        const uint64_t t = alloc(len);
        p.steps.push_back(mkStep(GLOO_HIP_STEP_COPY, -1, 0, GLOO_HIP_DST_ARENA, t, J.elem, len));
        leafAt[rank] = {GLOO_HIP_SRC_ARENA, t};
      } else {
        leafAt[rank] = {leafFlags, J.elem};
      }
      auto src = [&](int leaf) {
        const auto& l = leafAt.at(leaf);
        return mkStep(GLOO_HIP_STEP_FOLD_SRC, -1, 0, l.first, 0, l.second, len);
      };
      std::vector<int> order;
      if (leftChain(F, J.tree, order)) {
        for (int l : order) p.steps.push_back(src(l));
        p.steps.push_back(mkStep(GLOO_HIP_STEP_FOLD, -1, 0, 0, J.lo, 0, len));
      } else if (order.clear(), rightChain(F, J.tree, order)) {
        for (int l : order) p.steps.push_back(src(l));
        p.steps.push_back(mkStep(GLOO_HIP_STEP_FOLD, -1, 0, GLOO_HIP_FOLD_REVERSE, J.lo, 0, len));
      } else if (order.clear(), balanced(F, J.tree, order) > 0) {
        for (int l : order) p.steps.push_back(src(l));
        p.steps.push_back(mkStep(GLOO_HIP_STEP_FOLD, -1, 0, GLOO_HIP_FOLD_TREE, J.lo, 0, len));
      } else {
        // any other shape: post-order, one pairwise fold per node, inner
        // nodes into arena temporaries
        std::function<std::pair<int, uint64_t>(int, bool)> eval = [&](int t, bool root) {
          const TreeNode& n = F.at(t);
          if (n.leaf >= 0) return leafAt.at(n.leaf);
          const auto a = eval(n.lhs, false);
          const auto b = eval(n.rhs, false);
          p.steps.push_back(mkStep(GLOO_HIP_STEP_FOLD_SRC, -1, 0, a.first, 0, a.second, len));
          p.steps.push_back(mkStep(GLOO_HIP_STEP_FOLD_SRC, -1, 0, b.first, 0, b.second, len));
          if (root) {
            p.steps.push_back(mkStep(GLOO_HIP_STEP_FOLD, -1, 0, 0, J.lo, 0, len));
            return std::make_pair(0, J.lo);
          }
          const uint64_t tmp = alloc(len);
          p.steps.push_back(mkStep(GLOO_HIP_STEP_FOLD, -1, 0, GLOO_HIP_DST_ARENA, tmp, 0, len));
          return std::make_pair((int)GLOO_HIP_SRC_ARENA, tmp);
        };
        eval(J.tree, true);
      }
    }
    if (!allreduce)
      for (int s : peersFrom(rank)) p.steps.push_back(mkStep(GLOO_HIP_STEP_NOTIFY, s, GLOO_HIP_SLOT_NOTIFY));
    if (toRoot && rank != ns->root) {
      // results to the root; its previous-run copy-out must be done
      p.steps.push_back(mkStep(GLOO_HIP_STEP_WAIT_NOTIFY, ns->root, GLOO_HIP_SLOT_DIST_NOTIFY, GLOO_HIP_PREV_RUN));
      for (int j : byOwner[rank])
        p.steps.push_back(mkStep(GLOO_HIP_STEP_SEND, ns->root, slotOf(j, GLOO_HIP_SLOT_AUX0), 0, 0, jobs[j].lo,
                                 jobs[j].hi - jobs[j].lo));
    }
    if (allreduce)
      for (int j : byOwner[rank])
        for (int s : peersFrom(rank))
          p.steps.push_back(mkStep(GLOO_HIP_STEP_SEND, s, slotOf(j, GLOO_HIP_SLOT_AUX0), 0, 0, jobs[j].lo,
                                   jobs[j].hi - jobs[j].lo));
  }
  if (toRoot && rank == ns->root) {
    for (int o : peersFrom(rank))
      for (int j : byOwner[o]) p.steps.push_back(mkStep(GLOO_HIP_STEP_WAIT_RECV, o, slotOf(j, GLOO_HIP_SLOT_AUX0)));
    for (int o : peersFrom(rank))
      for (int j : byOwner[o])
        p.steps.push_back(mkStep(GLOO_HIP_STEP_COPY, -1, 0, GLOO_HIP_SRC_ARENA, jobs[j].lo, rootRegion[j],
                                 jobs[j].hi - jobs[j].lo));
    for (int o : peersFrom(rank))
      if (!byOwner[o].empty()) p.steps.push_back(mkStep(GLOO_HIP_STEP_NOTIFY, o, GLOO_HIP_SLOT_DIST_NOTIFY));
  }
  if (allreduce) {
    for (int o : peersFrom(rank))
      for (int j : byOwner[o]) p.steps.push_back(mkStep(GLOO_HIP_STEP_WAIT_RECV, o, slotOf(j, GLOO_HIP_SLOT_AUX0)));
    for (int o : peersFrom(rank))
      for (int j : byOwner[o])
        p.steps.push_back(mkStep(GLOO_HIP_STEP_COPY, -1, 0, GLOO_HIP_SRC_ARENA, jobs[j].lo, agRegion[j],
                                 jobs[j].hi - jobs[j].lo));
    if (nptrs > 1) p.steps.push_back(mkStep(GLOO_HIP_STEP_LOCAL_BCAST, -1, 0, 0, 0, 0, count));
  }
  p.arena = top;
  return p;
}

}  // namespace gloo_amd

// Branch-and-bound level kernels (K9): close / flag / split nodes into the next BFS level.
//
// fa_split_kernel      one wave64 per node of a sub-batch: drop closed nodes and nodes of decided
//                      partitions; flag possible violations for exact host confirmation (every
//                      possible PA pair of a leaf = single lattice point; the LP-optimal vertex
//                      pair of an inner node); split open inner nodes along their top-m scored
//                      dimensions into 2^m children, enforcing the per-partition node budget and
//                      the pool capacity with device atomics (overflow => partition UNKNOWN).
//                      Branching rule (per partition, so a partition's search tree does not depend
//                      on which other partitions share its chunk): a partition with w nodes in
//                      this level splits each along m = clamp(floor(log2(target / w)), 1, m_max)
//                      dimensions -- wide first levels, binary once its frontier reaches target.
//                      Relaxed queries keep a separate x' box for the relaxed features and
//                      tighten the |x_r - x'_r| <= tau coupling per child (empty children dropped).
//                      Budget (deterministic): a partition keeps splitting while its node count
//                      at the START of the level is below the budget (the last level may
//                      overshoot it); at the first level that starts at or over the budget its
//                      open nodes are bounded, their candidates emitted, and it goes to
//                      ST_STOPPING; fa_settle turns it UNKNOWN with open_left = its open inner
//                      nodes of that level.  No decision depends on the order in which device
//                      atomics were served (concurrent streams, other GPUs, rank counts).
// fa_settle            level end: STOPPING -> UNKNOWN (+ open_left), next level's budget reference,
//                      level counters to pinned host memory, next counter slot cleared.
// fa_mark_unknown      time budget hit: every RUNNING partition with live nodes -> UNKNOWN.
// fa_set_status        host-confirmed SAT partitions -> SAT.
#include <algorithm>

#include "args.h"

#define ST_UNKNOWN 0
#define ST_SAT 1
#define ST_UNSAT 2
#define ST_RUNNING 3
#define ST_STOPPING 4   // out of budget during the current level

// budget / capacity exhausted: the partition ends UNKNOWN with this node left open
__device__ __forceinline__ void fa_stop(const SplitArgs& a, int p) { a.status[p] = ST_STOPPING; }

// Dimension d of child c (bit j of c = upper half along dims[j]): x box [lo, hi], x' box [plo, phi].
// Every dimension of a child is a function of that dimension alone (the relaxed |x_r - x'_r| <= tau
// tightening included), so lanes can build (child, dim) entries independently.
__device__ __forceinline__ void fa_child_dim(const SplitArgs& a, const float* xl, const float* xh, const float* pl,
                                             const float* ph, const int* dims, int m, int c, int d, float& lo,
                                             float& hi, float& plo, float& phi) {
  lo = xl[d]; hi = xh[d]; plo = pl[d]; phi = ph[d];
  for (int j = 0; j < m; ++j) {
    const int dd = dims[j];
    const bool up = (c >> j) & 1;
    if (dd == d) {
      const float mid = floorf(0.5f * (xl[d] + xh[d]));
      if (up) lo = mid + 1.f; else hi = mid;
      if (a.relaxed && a.shared[d]) { plo = lo; phi = hi; }
    } else if (dd == a.n0 + d) {
      const float mid = floorf(0.5f * (pl[d] + ph[d]));
      if (up) plo = mid + 1.f; else phi = mid;
    }
  }
  if (a.relaxed)
    for (int k = 0; k < a.nra; ++k)
      if (a.ra_idx[k] == d) {
        plo = fmaxf(plo, lo - a.tau);
        phi = fminf(phi, hi + a.tau);
        lo = fmaxf(lo, plo - a.tau);
        hi = fminf(hi, phi + a.tau);
      }
}

// (score, dim) arg-max over the wave: larger score wins, ties go to the lower dimension (the
// sequential scan's first strict maximum)
__device__ __forceinline__ void fa_wave_argmax(float& s, int& d) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float s2 = __shfl_xor(s, o);
    const int d2 = __shfl_xor(d, o);
    if (s2 > s || (s2 == s && d2 < d)) { s = s2; d = d2; }
  }
}

__device__ __forceinline__ void fa_settle_counters(const SettleArgs& s) {
  // level counters straight into pinned host memory (no blit per level), next slot cleared; the
  // counters were accumulated by device atomics (L2): read them the same way
  const int c0 = __hip_atomic_load(&s.counters_cur[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const int c1 = __hip_atomic_load(&s.counters_cur[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(&s.host_counts[0], c0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(&s.host_counts[1], c1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  s.counters_next[0] = 0;
  s.counters_next[1] = 0;
}

__device__ __forceinline__ void fa_settle_part(const SettleArgs& s, int p) {
  const int8_t st = s.status[p];
  if (st == ST_STOPPING) {
    s.status[p] = ST_UNKNOWN;
    if (s.part_open) s.part_open[p] = s.lvl_open[p];
  } else if (s.prob && s.prob[p] && st == ST_RUNNING) {
    // stepped escalation: budget -> esc.budget[0] -> ... -> budget2; at each step's probation
    // level the frontier must be at most max_open (first step) / esc.open[k-1] (step k)
    const int cur = s.pbudget[p];
    int k = 0;
    while (k < s.esc.n && s.esc.budget[k] <= cur) ++k;
    const int thr = k == 0 ? s.max_open : s.esc.open[k - 1];
    if (s.lvl_open[p] <= thr) {
      s.pbudget[p] = k < s.esc.n ? s.esc.budget[k] : s.budget2;
    } else {
      s.status[p] = ST_UNKNOWN;
      if (s.part_open) s.part_open[p] = s.lvl_open[p];
    }
  }
  if (s.prob) s.prob[p] = 0;
  s.lvl_open[p] = 0;
  s.prev_start[p] = s.nodes_start[p];
  s.nodes_start[p] = s.part_nodes[p];     // the next level's budget reference
}

// Per-node plan of the split kernel (phase A -> phase C through LDS).
struct FaSplitPlan {
  unsigned long long fmask;   // feasible children (bit c = child c)
  unsigned long long dims;    // split dims, 7 bits each
  int m;                      // split dim count (children = 2^m before feasibility)
  int nchild;                 // feasible children to write
  int ncand;                  // candidate pairs to write
  int leaf;
  int part;                   // partition of an open inner node (-1: nothing to count)
};

// Possible-violation test of (orientation, pair) t at a leaf node (rows of the node's PA values).
__device__ __forceinline__ bool fa_leaf_poss(const SplitArgs& a, int n, int t) {
  const int o = t / a.Pp, q = t - o * a.Pp;
  const size_t ri = (size_t)n * a.V + (int)a.pairs[2 * q], rj = (size_t)n * a.V + (int)a.pairs[2 * q + 1];
  return (o == 0) ? (a.olb[ri] < 0.f && a.oubp[rj] > 0.f) : (a.oub[ri] > 0.f && a.olbp[rj] < 0.f);
}

// Inclusive wave64 prefix sum.
__device__ __forceinline__ int fa_wave_incl_scan(int v, int lane) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int u = __shfl_up(v, o);
    if (lane >= o) v += u;
  }
  return v;
}

// One wave64 per node, npw (1..FA_SPLIT_NPW) nodes per wave, FA_SPLIT_WAVES * npw nodes per
// workgroup (npw shrinks for small levels: a wave walks its nodes one after another, so at a 1/8
// shard's small levels 8 nodes per wave made the kernel 8 dependent node latencies long), three phases:
//   A  each wave plans its nodes: split dims by wave arg-max reductions, feasible children by a
//      ballot (lane c = child c), candidate counts by ballots over the leaf's PA pairs;
//   B  wave 0 scans the block's child / candidate counts and reserves both ranges with ONE
//      atomic each (a per-node atomic on the level counter serialised ~32 K same-address atomics
//      per sub-batch in L2: ~135 us of the kernel's time in the round-2 baseline), and adds the
//      per-partition counters (open inner nodes of the level, children made) with one atomic
//      per run of equal partitions among the block's 64 nodes -- a partition's nodes are
//      contiguous in the pool, so a deep partition no longer sends one same-address atomic per
//      node to L2;
//   C  each wave writes its children lane-parallel over (child, dim) entries (consecutive lanes
//      store consecutive floats of the pool) and its candidate pairs.
#define FA_SPLIT_WAVES 8
#define FA_SPLIT_NPW 8
#define FA_SPLIT_NB (FA_SPLIT_WAVES * FA_SPLIT_NPW)
__global__ void __launch_bounds__(64 * FA_SPLIT_WAVES) fa_split_kernel(SplitArgs a, int npw) {
  __shared__ FaSplitPlan plan[FA_SPLIT_NB];
  __shared__ int child_off[FA_SPLIT_NB], cand_off[FA_SPLIT_NB];
  // per-node scalars of the block's 64 nodes, fetched once by 64 threads in parallel: each wave
  // then walks its 8 nodes from LDS instead of paying the dependent chain node -> partition ->
  // status / budget reference (4 global round trips) once per node
  __shared__ int s_part[FA_SPLIT_NB], s_ns[FA_SPLIT_NB], s_ws[FA_SPLIT_NB], s_bud[FA_SPLIT_NB];
  __shared__ float s_pe[FA_SPLIT_NB][4];
  __shared__ int8_t s_st[FA_SPLIT_NB];
  __shared__ uint8_t s_open[FA_SPLIT_NB], s_leaf[FA_SPLIT_NB];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int n0 = a.n0;
  const int npair = a.norient * a.Pp;
  const int nb = FA_SPLIT_WAVES * npw;             // nodes of this workgroup (<= FA_SPLIT_NB)
  if (threadIdx.x >= nb && threadIdx.x < FA_SPLIT_NB) plan[threadIdx.x] = FaSplitPlan{0ull, 0ull, 0, 0, 0, 0, -1};
  if (threadIdx.x < nb) {
    const int t = threadIdx.x;
    const int n = blockIdx.x * nb + t;
    uint8_t op = 0;
    int p = 0;
    if (n < a.Nn) {
      op = a.open[n];
      p = a.part[n];
      s_leaf[t] = a.leaf[n];
      s_pe[t][0] = a.pe_lb[n];
      s_pe[t][1] = a.pe_ub[n];
      s_pe[t][2] = a.pe_lb[a.Nn + n];
      s_pe[t][3] = a.pe_ub[a.Nn + n];
    }
    s_open[t] = op;
    s_part[t] = p;
    if (op) {
      s_st[t] = a.status[p];
      s_ns[t] = a.nodes_start[p];
      s_ws[t] = a.nodes_start[p] - a.prev_start[p];
      s_bud[t] = a.pbudget ? a.pbudget[p] : a.budget;
    }
  }
  __syncthreads();
  // ---------------- phase A: plan
  for (int i = 0; i < npw; ++i) {
    const int loc = wave * npw + i;
    const int n = blockIdx.x * nb + loc;
    FaSplitPlan pl{0ull, 0ull, 0, 0, 0, 0, -1};
    do {
      if (n >= a.Nn || !s_open[loc]) break;                // wave-uniform
      const int p = s_part[loc];
      // RUNNING or STOPPING (budget ran out earlier in this same level): both still active
      const int8_t s0 = s_st[loc];
      if (s0 != ST_RUNNING && s0 != ST_STOPPING) break;
      if (s_leaf[loc]) {   // every possible PA pair of the single lattice point goes to the host check
        pl.leaf = 1;
        for (int t0 = 0; t0 < npair; t0 += 64)
          pl.ncand += __popcll(__ballot(t0 + lane < npair && fa_leaf_poss(a, n, t0 + lane)));
        break;
      }
      pl.part = p;   // counted in phase B: one open inner node of p in this level
      {
        const float lbx = s_pe[loc][0], ubx = s_pe[loc][1];
        const float lbp = s_pe[loc][2], ubp = s_pe[loc][3];
        pl.ncand = ((lbx < 0.f && ubp > 0.f) || (ubx > 0.f && lbp < 0.f)) ? 1 : 0;
      }
      // split along the top-m scored dimensions (2 n0 <= 128 scores: two per lane)
      const float* sc = a.scores + (size_t)n * 2 * n0;
      int mreq = 1;
      {
        const int mmax = a.m < FA_MAX_SPLIT ? a.m : FA_MAX_SPLIT;
        const int w = s_ws[loc];                           // this partition's nodes in the level
        while (mreq < mmax && ((long long)w << (mreq + 1)) <= (long long)a.target) ++mreq;
      }
      const int d0 = lane, d1 = lane + 64;
      float s0v = (d0 < 2 * n0) ? sc[d0] : -1.f;
      float s1v = (d1 < 2 * n0) ? sc[d1] : -1.f;
      if (!(s0v > -0.5f)) s0v = -1.f;                      // NaN / below the threshold: never picked
      if (!(s1v > -0.5f)) s1v = -1.f;
      int dims[FA_MAX_SPLIT];
      int m = 0;
      for (int j = 0; j < mreq; ++j) {
        float sv = s0v >= s1v ? s0v : s1v;                 // ties: d0 < d1
        int d = s0v >= s1v ? d0 : d1;
        if (sv <= -0.5f) d = 0x7fffffff;
        fa_wave_argmax(sv, d);
        if (sv <= -0.5f) break;                            // wave-uniform after the reduction
        dims[m++] = d;
        if (d == d0) s0v = -1.f;
        if (d == d1) s1v = -1.f;
      }
      if (m == 0) break;   // no splittable dimension: treated as leaf by the certificate
      {
        const int bud = s_bud[loc];
        if (s_ns[loc] >= bud) {
          if (a.prob && bud < a.budget2) {
            // inline escalation: on probation this level (children are made); fa_settle keeps
            // it going with budget2 if its open frontier of this level is small, else UNKNOWN
            if (lane == 0) a.prob[p] = 1;
          } else {
            if (lane == 0) fa_stop(a, p);
            break;
          }
        }
      }
      const int k = 1 << m;
      const float* xl = a.xlo + (size_t)n * n0;
      const float* xh = a.xhi + (size_t)n * n0;
      const float* xpl = a.relaxed ? a.xplo + (size_t)n * n0 : xl;
      const float* xph = a.relaxed ? a.xphi + (size_t)n * n0 : xh;
      bool ok = lane < k;   // children feasibility (the relaxed coupling can empty a child)
      if (a.relaxed && ok)
        for (int d = 0; d < n0; ++d) {
          float lo, hi, plo, phi;
          fa_child_dim(a, xl, xh, xpl, xph, dims, m, lane, d, lo, hi, plo, phi);
          ok = ok && lo <= hi && plo <= phi;
        }
      pl.fmask = __ballot(ok);
      pl.nchild = __popcll(pl.fmask);
      pl.m = m;
      for (int j = 0; j < m; ++j) pl.dims |= (unsigned long long)dims[j] << (7 * j);
    } while (false);
    if (lane == 0) plan[loc] = pl;
  }
  __syncthreads();
  // ---------------- phase B: one reservation per workgroup for children and candidates
  if (wave == 0) {
    const int c = plan[lane].nchild, q = plan[lane].ncand;
    const int ci = fa_wave_incl_scan(c, lane), qi = fa_wave_incl_scan(q, lane);
    int cb = 0, qb = 0;
    if (lane == 63) {
      if (ci) cb = atomicAdd(a.count_out, ci);
      if (qi) qb = atomicAdd(a.cand_count, qi);
    }
    cb = __shfl(cb, 63);
    qb = __shfl(qb, 63);
    child_off[lane] = cb + ci - c;
    cand_off[lane] = qb + qi - q;
    // per-partition counters: segmented sums over runs of equal partition ids
    const int p = plan[lane].part;
    const int o = p >= 0 ? 1 : 0;
    const int oi = fa_wave_incl_scan(o, lane);
    const int pprev = __shfl_up(p, 1), pnext = __shfl_down(p, 1);
    const unsigned long long heads = __ballot(lane == 0 || pprev != p);
    const bool tail = lane == 63 || pnext != p;
    const int h = 63 - __clzll(heads & (lane == 63 ? ~0ull : ((2ull << lane) - 1ull)));
    const int ci_b = __shfl(ci, h > 0 ? h - 1 : 0), oi_b = __shfl(oi, h > 0 ? h - 1 : 0);
    if (tail && p >= 0) {
      const int so = oi - (h > 0 ? oi_b : 0), sc = ci - (h > 0 ? ci_b : 0);
      if (so && a.lvl_open) atomicAdd(&a.lvl_open[p], so);
      if (sc) atomicAdd(&a.part_nodes[p], sc);
    }
  }
  __syncthreads();
  // ---------------- phase C: write candidates and children
  for (int i = 0; i < npw; ++i) {
    const int loc = wave * npw + i;
    const int n = blockIdx.x * nb + loc;
    const FaSplitPlan pl = plan[loc];
    if (pl.ncand == 0 && pl.nchild == 0) continue;         // wave-uniform (LDS broadcast)
    const int p = s_part[loc];
    const float* xl = a.xlo + (size_t)n * n0;
    const float* xh = a.xhi + (size_t)n * n0;
    const float* xpl = a.relaxed ? a.xplo + (size_t)n * n0 : xl;
    const float* xph = a.relaxed ? a.xphi + (size_t)n * n0 : xh;
    if (pl.leaf) {
      int slot0 = cand_off[loc];
      for (int t0 = 0; t0 < npair; t0 += 64) {
        const int t = t0 + lane;
        const bool poss = t < npair && fa_leaf_poss(a, n, t);
        const unsigned long long bm = __ballot(poss);
        if (poss) {
          const int slot = slot0 + __popcll(bm & ((1ull << lane) - 1ull));
          if (slot >= a.cand_cap) {
            fa_stop(a, p);        // cannot confirm this leaf: stay sound
          } else {
            const int o = t / a.Pp, q = t - o * a.Pp;
            const int vi = (int)a.pairs[2 * q], vj = (int)a.pairs[2 * q + 1];
            float* cbuf = a.cand_buf + (size_t)slot * (2 * n0 + 1);
            for (int d = 0; d < n0; ++d) {
              cbuf[d] = xl[d];
              cbuf[n0 + d] = xpl[d];
            }
            for (int k = 0; k < a.npa; ++k) {
              cbuf[a.pa_idx[k]] = (float)a.values[vi * a.npa + k];
              cbuf[n0 + a.pa_idx[k]] = (float)a.values[vj * a.npa + k];
            }
            cbuf[2 * n0] = __int_as_float(p);
          }
        }
        slot0 += __popcll(bm);
      }
      continue;
    }
    if (pl.ncand) {
      const int slot = cand_off[loc];
      if (slot < a.cand_cap) {
        float* cbuf = a.cand_buf + (size_t)slot * (2 * n0 + 1);
        for (int d = lane; d < 2 * n0 + 1; d += 64)
          cbuf[d] = d < n0 ? a.cand_x[(size_t)n * n0 + d]
                           : (d < 2 * n0 ? a.cand_xp[(size_t)n * n0 + d - n0] : __int_as_float(p));
      }
    }
    if (pl.nchild == 0) continue;
    const int off = child_off[loc];
    if (off + pl.nchild > a.cap) {
      // pool full: the partition stops UNKNOWN.  Slots of this reservation below the capacity
      // are counted in the next level, so they get a copy of the parent (a sub-box of its own
      // partition: re-bounding it is redundant but sound) instead of stale or unset entries.
      if (lane == 0) fa_stop(a, p);
      const int lim = a.cap - off;
      for (int e = lane; e < lim * n0; e += 64) {
        const int r = e / n0, d = e - r * n0;
        const size_t o = (size_t)(off + r) * n0 + d;
        a.oxlo[o] = xl[d];
        a.oxhi[o] = xh[d];
        if (a.relaxed) { a.oxplo[o] = xpl[d]; a.oxphi[o] = xph[d]; }
      }
      for (int r = lane; r < lim; r += 64) a.opart[off + r] = p;
      continue;
    }
    int dims[FA_MAX_SPLIT];
    for (int j = 0; j < pl.m; ++j) dims[j] = (int)((pl.dims >> (7 * j)) & 127ull);
    // output slot of feasible child c = off + (feasible children before c)
    if ((pl.fmask >> lane) & 1ull) a.opart[off + __popcll(pl.fmask & ((1ull << lane) - 1ull))] = p;
    const int dense = (pl.fmask & (pl.fmask + 1ull)) == 0ull;   // feasible children = 0 .. nchild-1
    for (int e = lane; e < pl.nchild * n0; e += 64) {
      const int r = e / n0, d = e - r * n0;      // r-th feasible child
      int c = r;
      if (!dense) {                              // relaxed: the r-th set bit of fmask
        unsigned long long mm = pl.fmask;
        for (int t = 0; t < r; ++t) mm &= mm - 1ull;
        c = __ffsll((long long)mm) - 1;
      }
      float lo, hi, plo, phi;
      fa_child_dim(a, xl, xh, xpl, xph, dims, pl.m, c, d, lo, hi, plo, phi);
      const size_t o = (size_t)(off + r) * n0 + d;
      a.oxlo[o] = lo;
      a.oxhi[o] = hi;
      if (a.relaxed) {
        a.oxplo[o] = plo;
        a.oxphi[o] = phi;
      }
    }
  }
  // ---------------- fused level end (the level's last sub-batch): the last workgroup to finish
  // settles every partition -- one launch per level less.  Release this workgroup's writes, count
  // it done; the last one acquires everything (the fence invalidates its L1) and settles.
  if (a.settle.P > 0) {
    __shared__ int s_last;
    __threadfence();
    __syncthreads();
    if (threadIdx.x == 0) s_last = atomicAdd(a.settle.done, 1) == (int)gridDim.x - 1;
    __syncthreads();
    if (s_last) {
      __threadfence();
      if (threadIdx.x == 0) fa_settle_counters(a.settle);
      for (int p = threadIdx.x; p < a.settle.P; p += blockDim.x) fa_settle_part(a.settle, p);
      if (threadIdx.x == 0) *a.settle.done = 0;   // ready for the next fused launch (stream order)
    }
  }
}

// Solve start, one launch: per-partition state from the staged host block [status int8 x P,
// padded to 4 B | running partition ids x n_run | lo x n_run*n0 | hi x n_run*n0] (one H2D copy),
// the root node pool (x' boxes widened by tau on the relaxed dims), the level counters.
__global__ void fa_bab_init_kernel(BabInitArgs a) {
  const int tid = blockIdx.x * FA_THREADS + threadIdx.x;
  const int nth = gridDim.x * FA_THREADS;
  const int8_t* st = reinterpret_cast<const int8_t*>(a.stage);
  const int* run = reinterpret_cast<const int*>(a.stage + ((a.P + 3) & ~3));
  const float* lo = reinterpret_cast<const float*>(run + a.n_run);
  const float* hi = lo + (size_t)a.n_run * a.n0;
  for (int p = tid; p < a.P; p += nth) {
    a.status[p] = st[p];
    a.nodes[p] = 0;
    a.open_left[p] = 0;
    a.lvl_open[p] = 0;
    a.nodes_start[p] = 0;
    a.prev_start[p] = -1;      // one root node in the first level
    if (a.pbudget) a.pbudget[p] = a.budget;
    if (a.prob) a.prob[p] = 0;
  }
  for (int i = tid; i < a.n_run; i += nth) a.part[i] = run[i];
  const size_t ne = (size_t)a.n_run * a.n0;
  for (size_t e = tid; e < ne; e += nth) {
    a.xlo[e] = lo[e];
    a.xhi[e] = hi[e];
    if (a.xplo) {
      const int d = (int)(e % a.n0);
      bool r = false;
      for (int k = 0; k < a.nra; ++k) r |= a.ra_idx[k] == d;
      a.xplo[e] = r ? lo[e] - a.tau : lo[e];
      a.xphi[e] = r ? hi[e] + a.tau : hi[e];
    }
  }
  if (tid < 5) a.counters[tid] = 0;   // two level-counter slots + the fused settle's workgroup counter
}

// Solve end, one launch: status / nodes / open_left packed into one int block (one D2H copy).
__global__ void fa_bab_finish_kernel(int P, const int8_t* status, const int* nodes, const int* open_left, int* out) {
  const int p = blockIdx.x * FA_THREADS + threadIdx.x;
  if (p >= P) return;
  out[p] = status[p];
  out[P + p] = nodes[p];
  out[2 * P + p] = open_left[p];
}

__global__ void fa_mark_unknown_kernel(const int* part, int n, int8_t* status) {
  const int i = blockIdx.x * FA_THREADS + threadIdx.x;
  if (i >= n) return;
  const int p = part[i];
  if (status[p] == ST_RUNNING || status[p] == ST_STOPPING) status[p] = ST_UNKNOWN;
}

// Inline escalation (prob != nullptr): a partition that started this level at its first budget
// was on probation (its nodes bounded, candidates emitted, children made).  If its open inner
// nodes of this level are at most max_open it continues with budget2 -- the deeper second pass
// of the two-pass schedule, same selection rule (profiles/escalate_sweep/), without restarting
// from the root; otherwise it ends UNKNOWN with open_left = those nodes, exactly like the
// first pass.  Its surplus children are skipped by the bound kernels (status filter).
__global__ void fa_settle_kernel(SettleArgs s) {
  const int p = blockIdx.x * FA_THREADS + threadIdx.x;
  if (p == 0) fa_settle_counters(s);
  if (p < s.P) fa_settle_part(s, p);
}

__global__ void fa_set_status_kernel(const int* idx, int n, int8_t* status, int8_t v) {
  const int i = blockIdx.x * FA_THREADS + threadIdx.x;
  if (i < n) status[idx[i]] = v;
}

extern "C" int fa_split_launch(SplitArgs a, hipStream_t stream) {
  if (a.Nn <= 0) return 0;
  if (a.nra > FA_MAX_RA || a.npa > FA_CMAX_PA || a.n0 > 64) return -3;
  // nodes per wave: 8 while that still makes >= 1024 workgroups (4 per CU), fewer for small levels
  int npw = FA_SPLIT_NPW;
  while (npw > 1 && (a.Nn + FA_SPLIT_WAVES * npw - 1) / (FA_SPLIT_WAVES * npw) < 1024) npw >>= 1;
  const int nb = FA_SPLIT_WAVES * npw;
  hipLaunchKernelGGL(fa_split_kernel, dim3((a.Nn + nb - 1) / nb), dim3(64 * FA_SPLIT_WAVES), 0, stream, a, npw);
  return (int)hipGetLastError();
}

extern "C" int fa_mark_unknown_launch(const int* part, int n, int8_t* status, hipStream_t stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(fa_mark_unknown_kernel, dim3((n + FA_THREADS - 1) / FA_THREADS), dim3(FA_THREADS), 0, stream,
                     part, n, status);
  return (int)hipGetLastError();
}

extern "C" int fa_set_status_launch(const int* idx, int n, int8_t* status, int8_t v, hipStream_t stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(fa_set_status_kernel, dim3((n + FA_THREADS - 1) / FA_THREADS), dim3(FA_THREADS), 0, stream, idx,
                     n, status, v);
  return (int)hipGetLastError();
}

extern "C" int fa_settle_launch(SettleArgs s, hipStream_t stream) {
  const int n = s.P > 0 ? s.P : 1;
  hipLaunchKernelGGL(fa_settle_kernel, dim3((n + FA_THREADS - 1) / FA_THREADS), dim3(FA_THREADS), 0, stream, s);
  return (int)hipGetLastError();
}

extern "C" int fa_bab_init_launch(BabInitArgs a, hipStream_t stream) {
  if (a.nra > FA_MAX_RA) return -3;
  const long long work = std::max<long long>(std::max(a.P, a.n_run), (long long)a.n_run * a.n0);
  const int blocks = (int)std::min<long long>((work + FA_THREADS - 1) / FA_THREADS + 1, 4096);
  hipLaunchKernelGGL(fa_bab_init_kernel, dim3(blocks), dim3(FA_THREADS), 0, stream, a);
  return (int)hipGetLastError();
}

extern "C" int fa_bab_finish_launch(int P, const int8_t* status, const int* nodes, const int* open_left, int* out,
                                    hipStream_t stream) {
  if (P <= 0) return 0;
  hipLaunchKernelGGL(fa_bab_finish_kernel, dim3((P + FA_THREADS - 1) / FA_THREADS), dim3(FA_THREADS), 0, stream, P,
                     status, nodes, open_left, out);
  return (int)hipGetLastError();
}

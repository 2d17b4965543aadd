// Branch-and-bound level kernels (K9): close / flag / split nodes into the next BFS level.
//
// fa_split_kernel      one thread per node of a sub-batch: drop closed nodes and nodes of decided
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
#include "args.h"

#define ST_UNKNOWN 0
#define ST_SAT 1
#define ST_UNSAT 2
#define ST_RUNNING 3
#define ST_STOPPING 4   // out of budget during the current level

__device__ __forceinline__ void fa_tighten(const SplitArgs& a, float* lo, float* hi, float* plo, float* phi) {
  for (int k = 0; k < a.nra; ++k) {
    const int r = a.ra_idx[k];
    plo[r] = fmaxf(plo[r], lo[r] - a.tau);
    phi[r] = fminf(phi[r], hi[r] + a.tau);
    lo[r] = fmaxf(lo[r], plo[r] - a.tau);
    hi[r] = fminf(hi[r], phi[r] + a.tau);
  }
}

// budget / capacity exhausted: the partition ends UNKNOWN with this node left open
__device__ __forceinline__ void fa_stop(const SplitArgs& a, int p) { a.status[p] = ST_STOPPING; }

#define FA_SPLIT_THREADS 64
__global__ void __launch_bounds__(FA_SPLIT_THREADS) fa_split_kernel(SplitArgs a) {
  const int n = blockIdx.x * FA_SPLIT_THREADS + threadIdx.x;
  if (n >= a.Nn) return;
  const int p = a.part[n];
  if (!a.open[n]) return;
  // RUNNING or STOPPING (budget ran out earlier in this same level): both still active this level
  const int8_t s0 = a.status[p];
  if (s0 != ST_RUNNING && s0 != ST_STOPPING) return;
  if (!a.leaf[n] && a.lvl_open) atomicAdd(&a.lvl_open[p], 1);
  const int n0 = a.n0;
  const float* xl = a.xlo + (size_t)n * n0;
  const float* xh = a.xhi + (size_t)n * n0;
  const float* pl = a.relaxed ? a.xplo + (size_t)n * n0 : xl;
  const float* ph = a.relaxed ? a.xphi + (size_t)n * n0 : xh;
  // ---------------- candidates for exact confirmation
  if (a.leaf[n]) {
    for (int o = 0; o < a.norient; ++o)
      for (int q = 0; q < a.Pp; ++q) {
        const int vi = (int)a.pairs[2 * q], vj = (int)a.pairs[2 * q + 1];
        const size_t ri = (size_t)n * a.V + vi, rj = (size_t)n * a.V + vj;
        const bool poss = (o == 0) ? (a.olb[ri] < 0.f && a.oubp[rj] > 0.f) : (a.oub[ri] > 0.f && a.olbp[rj] < 0.f);
        if (!poss) continue;
        const int slot = atomicAdd(a.cand_count, 1);
        if (slot >= a.cand_cap) {      // cannot confirm this leaf: stay sound
          fa_stop(a, p);
          return;
        }
        float* cb = a.cand_buf + (size_t)slot * 2 * n0;
        for (int d = 0; d < n0; ++d) {
          cb[d] = xl[d];
          cb[n0 + d] = pl[d];
        }
        for (int k = 0; k < a.npa; ++k) {
          cb[a.pa_idx[k]] = (float)a.values[vi * a.npa + k];
          cb[n0 + a.pa_idx[k]] = (float)a.values[vj * a.npa + k];
        }
        a.cand_part[slot] = p;
      }
    return;  // a leaf is decided by the host check
  }
  {
    const float lbx = a.pe_lb[n], ubx = a.pe_ub[n];
    const float lbp = a.pe_lb[a.Nn + n], ubp = a.pe_ub[a.Nn + n];
    const bool poss = (lbx < 0.f && ubp > 0.f) || (ubx > 0.f && lbp < 0.f);
    if (poss) {
      const int slot = atomicAdd(a.cand_count, 1);
      if (slot < a.cand_cap) {
        float* cb = a.cand_buf + (size_t)slot * 2 * n0;
        for (int d = 0; d < n0; ++d) {
          cb[d] = a.cand_x[(size_t)n * n0 + d];
          cb[n0 + d] = a.cand_xp[(size_t)n * n0 + d];
        }
        a.cand_part[slot] = p;
      }
    }
  }
  // ---------------- split along the top-m scored dimensions
  const float* sc = a.scores + (size_t)n * 2 * n0;
  int dims[FA_MAX_SPLIT];
  int m = 0;
  int mreq = 1;
  {
    const int mmax = a.m < FA_MAX_SPLIT ? a.m : FA_MAX_SPLIT;
    const int w = a.nodes_start[p] - a.prev_start[p];      // this partition's nodes in the level
    while (mreq < mmax && ((long long)w << (mreq + 1)) <= (long long)a.target) ++mreq;
  }
  for (int j = 0; j < mreq; ++j) {
    float best = -0.5f;
    int bd = -1;
    for (int d = 0; d < 2 * n0; ++d) {
      bool used = false;
      for (int u = 0; u < m; ++u) used |= (dims[u] == d);
      if (!used && sc[d] > best) { best = sc[d]; bd = d; }
    }
    if (bd < 0) break;
    dims[m++] = bd;
  }
  if (m == 0) return;  // no splittable dimension: treated as leaf by the certificate
  const int k = 1 << m;
  if (a.nodes_start[p] >= a.budget) { fa_stop(a, p); return; }
  if (!a.relaxed) {  // fast path: every child feasible, boxes written on the fly
    atomicAdd(&a.part_nodes[p], k);
    const int off = atomicAdd(a.count_out, k);
    if (off + k > a.cap) { fa_stop(a, p); return; }
    for (int c = 0; c < k; ++c) {
      float* ol = a.oxlo + (size_t)(off + c) * n0;
      float* oh = a.oxhi + (size_t)(off + c) * n0;
      for (int d = 0; d < n0; ++d) {
        float lo = xl[d], hi = xh[d];
        for (int j = 0; j < m; ++j)
          if (dims[j] == d) {
            const float mid = floorf(0.5f * (lo + hi));
            if ((c >> j) & 1) lo = mid + 1.f; else hi = mid;
          }
        ol[d] = lo;
        oh[d] = hi;
      }
      a.opart[off + c] = p;
    }
    return;
  }
  // children feasibility (relaxed coupling can empty a child)
  float clo[64], chi[64], cplo[64], cphi[64];
  if (n0 > 64) { fa_stop(a, p); return; }
  int feasible = 0;
  unsigned long long fmask = 0ull;
  for (int c = 0; c < k; ++c) {
    for (int d = 0; d < n0; ++d) { clo[d] = xl[d]; chi[d] = xh[d]; cplo[d] = pl[d]; cphi[d] = ph[d]; }
    for (int j = 0; j < m; ++j) {
      const int d = dims[j];
      const int bit = (c >> j) & 1;
      if (d < n0) {
        const float mid = floorf(0.5f * (xl[d] + xh[d]));
        if (bit) clo[d] = mid + 1.f; else chi[d] = mid;
        if (a.relaxed && a.shared[d]) { cplo[d] = clo[d]; cphi[d] = chi[d]; }
      } else {
        const int e = d - n0;
        const float mid = floorf(0.5f * (pl[e] + ph[e]));
        if (bit) cplo[e] = mid + 1.f; else cphi[e] = mid;
      }
    }
    bool ok = true;
    if (a.relaxed) {
      fa_tighten(a, clo, chi, cplo, cphi);
      for (int d = 0; d < n0; ++d) ok &= (clo[d] <= chi[d]) && (cplo[d] <= cphi[d]);
    }
    if (ok) { fmask |= (1ull << c); ++feasible; }
  }
  if (feasible == 0) return;
  atomicAdd(&a.part_nodes[p], feasible);
  const int off = atomicAdd(a.count_out, feasible);
  if (off + feasible > a.cap) { fa_stop(a, p); return; }
  int w = off;
  for (int c = 0; c < k; ++c) {
    if (!((fmask >> c) & 1ull)) continue;
    for (int d = 0; d < n0; ++d) { clo[d] = xl[d]; chi[d] = xh[d]; cplo[d] = pl[d]; cphi[d] = ph[d]; }
    for (int j = 0; j < m; ++j) {
      const int d = dims[j];
      const int bit = (c >> j) & 1;
      if (d < n0) {
        const float mid = floorf(0.5f * (xl[d] + xh[d]));
        if (bit) clo[d] = mid + 1.f; else chi[d] = mid;
        if (a.relaxed && a.shared[d]) { cplo[d] = clo[d]; cphi[d] = chi[d]; }
      } else {
        const int e = d - n0;
        const float mid = floorf(0.5f * (pl[e] + ph[e]));
        if (bit) cplo[e] = mid + 1.f; else cphi[e] = mid;
      }
    }
    if (a.relaxed) fa_tighten(a, clo, chi, cplo, cphi);
    float* ol = a.oxlo + (size_t)w * n0;
    float* oh = a.oxhi + (size_t)w * n0;
    for (int d = 0; d < n0; ++d) { ol[d] = clo[d]; oh[d] = chi[d]; }
    if (a.relaxed) {
      float* opl = a.oxplo + (size_t)w * n0;
      float* oph = a.oxphi + (size_t)w * n0;
      for (int d = 0; d < n0; ++d) { opl[d] = cplo[d]; oph[d] = cphi[d]; }
    }
    a.opart[w] = p;
    ++w;
  }
}

__global__ void fa_mark_unknown_kernel(const int* part, int n, int8_t* status) {
  const int i = blockIdx.x * FA_THREADS + threadIdx.x;
  if (i >= n) return;
  const int p = part[i];
  if (status[p] == ST_RUNNING || status[p] == ST_STOPPING) status[p] = ST_UNKNOWN;
}

__global__ void fa_settle_kernel(int P, int8_t* status, int* lvl_open, int* part_open, const int* part_nodes,
                                 int* nodes_start, int* prev_start, const int* counters_cur, int* counters_next,
                                 int* host_counts) {
  const int p = blockIdx.x * FA_THREADS + threadIdx.x;
  if (p == 0) {
    // level counters straight into pinned host memory (no blit per level), next slot cleared
    __hip_atomic_store(&host_counts[0], counters_cur[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(&host_counts[1], counters_cur[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    counters_next[0] = 0;
    counters_next[1] = 0;
  }
  if (p >= P) return;
  if (status[p] == ST_STOPPING) {
    status[p] = ST_UNKNOWN;
    if (part_open) part_open[p] = lvl_open[p];
  }
  lvl_open[p] = 0;
  prev_start[p] = nodes_start[p];
  nodes_start[p] = part_nodes[p];     // the next level's budget reference
}

__global__ void fa_set_status_kernel(const int* idx, int n, int8_t* status, int8_t v) {
  const int i = blockIdx.x * FA_THREADS + threadIdx.x;
  if (i < n) status[idx[i]] = v;
}

extern "C" int fa_split_launch(SplitArgs a, hipStream_t stream) {
  if (a.Nn <= 0) return 0;
  if (a.nra > FA_MAX_RA || a.npa > FA_CMAX_PA || a.n0 > 64) return -3;
  hipLaunchKernelGGL(fa_split_kernel, dim3((a.Nn + FA_SPLIT_THREADS - 1) / FA_SPLIT_THREADS), dim3(FA_SPLIT_THREADS),
                     0, stream, a);
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

extern "C" int fa_settle_launch(int P, int8_t* status, int* lvl_open, int* part_open, const int* part_nodes,
                                int* nodes_start, int* prev_start, const int* counters_cur, int* counters_next,
                                int* host_counts, hipStream_t stream) {
  const int n = P > 0 ? P : 1;
  hipLaunchKernelGGL(fa_settle_kernel, dim3((n + FA_THREADS - 1) / FA_THREADS), dim3(FA_THREADS), 0, stream, P,
                     status, lvl_open, part_open, part_nodes, nodes_start, prev_start, counters_cur, counters_next,
                     host_counts);
  return (int)hipGetLastError();
}

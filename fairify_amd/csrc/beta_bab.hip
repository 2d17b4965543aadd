// Device side of the native beta-CROWN branch-and-bound level loop (stage "beta"; host driver
// csrc/beta_runtime.cpp, torch reference engine/beta_bab.py).  The bounding itself is
// fa_beta_kernel (csrc/beta.hip); these kernels keep the node pool, the per-partition budgets and the
// probe on the device so a level costs one host synchronisation and one packed copy back:
//
//   count      -- per node: alive (partition RUNNING, relaxed x / x' boxes within tau); the partitions'
//                 node counts (budgets) are incremented for the whole level first, so no decision
//                 depends on the order the sub-batches run in; then per sub-batch its skip flags
//   rows       -- tightening rows of the children: x rows (PA = va) and x' rows (PA = vb, RA dims from
//                 x''s box) for the phase-aware symbolic + refine kernels (bounds.hip / refine.hip)
//   intersect  -- tightened bounds intersected with the inherited ones; an empty region closes the node
//   cand       -- candidate vertex pairs (x*, x'* with x'_r pulled into [x_r - tau, x_r + tau])
//   split      -- one wave per node: candidate records of open nodes whose rigorous point bounds allow a
//                 violation of their orientation (pinned host buffer), then 2 children (phase split with
//                 the parent's parameters and the monotone multiplier start, or input halving) or, past
//                 the partition's node budget, the partition stops
//   settle     -- trees with no node left are closed; a partition past its probe point with no closed
//                 tree stops (the probe of engine/beta_bab.py); the level counters go to the host
// The reference's Z3 loop this replaces: src/AC/Verify-AC.py:109-158 (one query per partition).
#include "args.h"
#include "common.h"

#define BB_UNKNOWN 0
#define BB_RUNNING 3
#define BB_STOPPING 4

namespace {

__global__ void fa_bb_count_kernel(BetaPoolArgs a) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= a.N) return;
  const int p = a.part[n];
  bool alive = a.status[p] == BB_RUNNING;
  if (alive && a.nra > 0) {       // relaxed: no admissible pair once x and x' boxes are > tau apart
    for (int k = 0; k < a.nra; ++k) {
      const int d = a.ra_idx[k];
      const size_t o = (size_t)n * a.n0 + d;
      if (a.plo[o] > a.hi[o] + a.tau || a.phi[o] < a.lo[o] - a.tau) alive = false;
    }
  }
  if (a.count) {
    if (alive) atomicAdd(&a.part_nodes[p], 1);
  } else {
    a.skip[n] = alive ? 0 : 1;
    if (a.root && !alive && a.diag) atomicAdd(a.diag + (a.status[p] == BB_RUNNING ? 1 : 0), 1);
  }
}

__global__ void fa_bb_rows_kernel(BetaPoolArgs a) {
  const long long tot = 2LL * a.N * a.n0;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < tot; e += (long long)gridDim.x * blockDim.x) {
    const int row = (int)(e / a.n0), d = (int)(e - (long long)row * a.n0);
    const int n = row >> 1, c = row & 1;
    const size_t o = (size_t)n * a.n0 + d;
    float lo = a.lo[o], hi = a.hi[o];
    if (c == 1 && a.nra > 0) {
      for (int k = 0; k < a.nra; ++k)
        if (a.ra_idx[k] == d) {
          lo = a.plo[o];
          hi = a.phi[o];
        }
    }
    for (int q = 0; q < a.npa; ++q)
      if (a.pa_idx[q] == d) lo = hi = (c == 0 ? a.va : a.vb)[(size_t)n * a.npa + q];
    a.rlo[(size_t)row * a.n0 + d] = lo;
    a.rhi[(size_t)row * a.n0 + d] = hi;
    if (d == 0) a.rpart[row] = a.part[n];
  }
}

__global__ void fa_bb_intersect_kernel(BetaPoolArgs a) {
  const long long tot = (long long)a.N * a.nh;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < tot; e += (long long)gridDim.x * blockDim.x) {
    const int n = (int)(e / a.nh), k = (int)(e - (long long)n * a.nh);
    if (a.skip[n]) continue;
    const size_t o = (size_t)n * a.nh + k;
    const size_t rA = (size_t)(2 * n) * a.nn + k, rB = (size_t)(2 * n + 1) * a.nn + k;
    a.LBA[o] = fmaxf(a.LBA[o], a.lay_lb[rA]);
    a.UBA[o] = fminf(a.UBA[o], a.lay_ub[rA]);
    a.LBB[o] = fmaxf(a.LBB[o], a.lay_lb[rB]);
    a.UBB[o] = fminf(a.UBB[o], a.lay_ub[rB]);
    if (k == 0 && (a.infeas[2 * n] || a.infeas[2 * n + 1])) a.skip[n] = 1;   // empty region: closed
  }
}

__global__ void fa_bb_cand_kernel(BetaPoolArgs a) {
  const long long tot = (long long)a.N * a.n0;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < tot; e += (long long)gridDim.x * blockDim.x) {
    const int n = (int)(e / a.n0), d = (int)(e - (long long)n * a.n0);
    const size_t o = (size_t)n * a.n0 + d;
    float xa = a.xstar[o];
    float xb = a.xpstar ? a.xpstar[o] : xa;
    for (int k = 0; k < a.nra; ++k)
      if (a.ra_idx[k] == d) xb = fminf(fmaxf(xb, xa - a.tau), xa + a.tau);
    for (int q = 0; q < a.npa; ++q)
      if (a.pa_idx[q] == d) {
        xa = a.va[(size_t)n * a.npa + q];
        xb = a.vb[(size_t)n * a.npa + q];
      }
    a.cpts[(size_t)(2 * n) * a.n0 + d] = xa;
    a.cpts[(size_t)(2 * n + 1) * a.n0 + d] = xb;
  }
}

// One wave64 per node (grid-stride over nodes).
__global__ void __launch_bounds__(FA_THREADS) fa_bb_split_kernel(BetaPoolArgs a) {
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int n0 = a.n0, nh = a.nh;
  for (int n = blockIdx.x * (FA_THREADS / 64) + wave; n < a.N; n += gridDim.x * (FA_THREADS / 64)) {
    if (a.skip[n]) continue;                                    // wave-uniform
    const double B = a.bound[n];
    if (B >= 0.0) continue;                                     // closed (+inf: empty)
    const int p = a.part[n];
    if (!(B < 0.0)) {
      // NaN: the node has no bound, so its tree cannot close -- the partition stops (UNKNOWN), never
      // counted as closed
      if (lane == 0) {
        a.status[p] = BB_STOPPING;
        if (a.nan_count) atomicAdd(a.nan_count, 1);
      }
      continue;
    }
    const int8_t st = a.status[p];
    if (st != BB_RUNNING && st != BB_STOPPING) continue;
    // ---- the concretising vertex pair, if its rigorous point bounds allow this orientation's violation
    const bool pos = a.osg[n] > 0;
    const bool poss = pos ? (a.pe_lb[2 * n] < 0.f && a.pe_ub[2 * n + 1] > 0.f)
                          : (a.pe_ub[2 * n] > 0.f && a.pe_lb[2 * n + 1] < 0.f);
    if (poss) {
      int slot = 0;
      if (lane == 0) slot = atomicAdd(a.cand_count, 1);
      slot = __shfl(slot, 0);
      if (slot < a.cand_cap) {
        float* cb = a.cand_buf + (size_t)slot * (2 * n0 + 1);
        for (int d = lane; d < 2 * n0 + 1; d += 64)
          cb[d] = d < n0 ? a.cpts[(size_t)(2 * n) * n0 + d]
                         : (d < 2 * n0 ? a.cpts[(size_t)(2 * n + 1) * n0 + d - n0] : __int_as_float(p));
      } else if (lane == 0) {
        a.status[p] = BB_STOPPING;                              // cannot confirm: stay sound
      }
    }
    const int sp = a.split[n];
    if (sp == a.leaf) continue;                                 // lattice leaf: the exact check decided
    if (st == BB_STOPPING || a.part_nodes[p] >= a.budget) {     // counted for this whole level
      if (lane == 0) a.status[p] = BB_STOPPING;
      continue;
    }
    int off = 0;
    if (lane == 0) off = atomicAdd(a.count_out, 2);
    off = __shfl(off, 0);
    if (off + 2 > a.cap) {                                      // pool full: the partition stops
      if (lane == 0) a.status[p] = BB_STOPPING;
      continue;
    }
    if (lane < 2) {
      a.opart[off + lane] = p;
      a.otree[off + lane] = a.tree[n];
      a.oosg[off + lane] = a.osg[n];
      a.ot[off + lane] = a.t[n];
    }
    if (lane == 0) atomicAdd(&a.tree_cnt[a.tree[n]], 2);
    // input split code -1 - d: x's dim d (d < n0) or x''s RA dim d - n0
    const int dsplit = sp < 0 ? -1 - sp : -1;
    for (int e = lane; e < 2 * n0; e += 64) {
      const int c = e / n0, d = e - c * n0;
      const size_t i = (size_t)n * n0 + d, oi = (size_t)(off + c) * n0 + d;
      float lo = a.lo[i], hi = a.hi[i];
      if (d == dsplit) {
        const float mid = floorf(0.5f * (lo + hi));
        if (c == 0) hi = mid; else lo = mid + 1.f;
      }
      a.olo[oi] = lo;
      a.ohi[oi] = hi;
      if (a.nra > 0) {
        float plo = a.plo[i], phi = a.phi[i];
        if (d + n0 == dsplit) {
          const float mid = floorf(0.5f * (plo + phi));
          if (c == 0) phi = mid; else plo = mid + 1.f;
        }
        a.oplo[oi] = plo;
        a.ophi[oi] = phi;
        if (a.gt) {
          a.ogt[(size_t)(off + c) * 2 * n0 + d] = a.gt[(size_t)n * 2 * n0 + d];
          a.ogt[(size_t)(off + c) * 2 * n0 + n0 + d] = a.gt[(size_t)n * 2 * n0 + n0 + d];
        }
      }
    }
    for (int e = lane; e < 2 * a.npa; e += 64) {
      const int c = e / a.npa, q = e - c * a.npa;
      a.ova[(size_t)(off + c) * a.npa + q] = a.va[(size_t)n * a.npa + q];
      a.ovb[(size_t)(off + c) * a.npa + q] = a.vb[(size_t)n * a.npa + q];
    }
    // neuron split: copy A neuron sp (< nh) or copy B neuron sp - nh; child 0 inactive, 1 active
    const int cfix = sp >= nh ? 1 : 0, kfix = sp >= 0 ? sp - cfix * nh : -1;
    for (int e = lane; e < 2 * nh; e += 64) {
      const int c = e / nh, k = e - c * nh;
      const size_t i = (size_t)n * nh + k, oi = (size_t)(off + c) * nh + k;
      a.oLBA[oi] = a.LBA[i];
      a.oUBA[oi] = a.UBA[i];
      a.oLBB[oi] = a.LBB[i];
      a.oUBB[oi] = a.UBB[i];
    }
    for (int e = lane; e < 2 * 2 * nh; e += 64) {          // phases [2][nh] per child
      const int c = e / (2 * nh), j = e - c * 2 * nh;     // j: copy * nh + k
      int8_t v = a.ph[(size_t)n * 2 * nh + j];
      if (kfix >= 0 && j == cfix * nh + kfix) v = c == 0 ? (int8_t)-1 : (int8_t)1;
      a.oph[(size_t)(off + c) * 2 * nh + j] = v;
    }
    for (int e = lane; e < 2 * 4 * nh; e += 64) {          // parameters [4][nh] per child
      const int c = e / (4 * nh), j = e - c * 4 * nh;
      float v = a.par[(size_t)n * 4 * nh + j];
      if (kfix >= 0 && j == (2 + cfix) * nh + kfix) v = a.warm_beta ? a.binit[2 * n + c] : 0.f;
      a.opar[(size_t)(off + c) * 4 * nh + j] = v;
    }
  }
}

// Trees with no node in the next pool are closed (count once per tree).
__global__ void fa_bb_settle_trees_kernel(int R0, const int* tree_cnt, uint8_t* tree_done, const int* tree_part,
                                          int* part_closed) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= R0) return;
  if (!tree_done[t] && tree_cnt[t] == 0) {
    tree_done[t] = 1;
    atomicAdd(&part_closed[tree_part[t]], 1);
  }
}

// Partitions: STOPPING -> UNKNOWN; the probe (past probe_at nodes with no closed tree: UNKNOWN);
// the level counters to the host (coherent pinned memory).
__global__ void fa_bb_settle_parts_kernel(int P, int8_t* status, const int* part_nodes, int probe_at,
                                          uint8_t* probed, const int* part_closed, int* probe_stops,
                                          const int* counters, int* host_counts) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p == 0) {
    __hip_atomic_store(&host_counts[0], counters[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(&host_counts[1], counters[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  if (p >= P) return;
  if (status[p] == BB_STOPPING) status[p] = BB_UNKNOWN;
  if (probe_at > 0 && status[p] == BB_RUNNING && !probed[p] && part_nodes[p] >= probe_at) {
    probed[p] = 1;
    if (part_closed[p] == 0) {
      status[p] = BB_UNKNOWN;
      atomicAdd(probe_stops, 1);
    }
  }
}

int grid_for(long long work, int per_block) {
  const long long b = (work + per_block - 1) / per_block;
  return (int)std::min<long long>(std::max<long long>(b, 1), 8192);
}

}  // namespace

extern "C" int fa_bb_count_launch(BetaPoolArgs a, hipStream_t s) {
  if (a.N <= 0) return 0;
  hipLaunchKernelGGL(fa_bb_count_kernel, dim3((a.N + FA_THREADS - 1) / FA_THREADS), dim3(FA_THREADS), 0, s, a);
  return (int)hipGetLastError();
}

extern "C" int fa_bb_rows_launch(BetaPoolArgs a, hipStream_t s) {
  if (a.N <= 0) return 0;
  hipLaunchKernelGGL(fa_bb_rows_kernel, dim3(grid_for(2LL * a.N * a.n0, FA_THREADS)), dim3(FA_THREADS), 0, s, a);
  return (int)hipGetLastError();
}

extern "C" int fa_bb_intersect_launch(BetaPoolArgs a, hipStream_t s) {
  if (a.N <= 0) return 0;
  hipLaunchKernelGGL(fa_bb_intersect_kernel, dim3(grid_for((long long)a.N * a.nh, FA_THREADS)), dim3(FA_THREADS), 0,
                     s, a);
  return (int)hipGetLastError();
}

extern "C" int fa_bb_cand_launch(BetaPoolArgs a, hipStream_t s) {
  if (a.N <= 0) return 0;
  hipLaunchKernelGGL(fa_bb_cand_kernel, dim3(grid_for((long long)a.N * a.n0, FA_THREADS)), dim3(FA_THREADS), 0, s, a);
  return (int)hipGetLastError();
}

extern "C" int fa_bb_split_launch(BetaPoolArgs a, hipStream_t s) {
  if (a.N <= 0) return 0;
  hipLaunchKernelGGL(fa_bb_split_kernel, dim3(grid_for(a.N, FA_THREADS / 64)), dim3(FA_THREADS), 0, s, a);
  return (int)hipGetLastError();
}

extern "C" int fa_bb_settle_launch(int R0, const int* tree_cnt, uint8_t* tree_done, const int* tree_part,
                                   int* part_closed, int P, int8_t* status, const int* part_nodes, int probe_at,
                                   uint8_t* probed, int* probe_stops, const int* counters, int* host_counts,
                                   hipStream_t s) {
  if (R0 > 0)
    hipLaunchKernelGGL(fa_bb_settle_trees_kernel, dim3((R0 + FA_THREADS - 1) / FA_THREADS), dim3(FA_THREADS), 0, s,
                       R0, tree_cnt, tree_done, tree_part, part_closed);
  const int np = P > 0 ? P : 1;
  hipLaunchKernelGGL(fa_bb_settle_parts_kernel, dim3((np + FA_THREADS - 1) / FA_THREADS), dim3(FA_THREADS), 0, s, P,
                     status, part_nodes, probe_at, probed, part_closed, probe_stops, counters, host_counts);
  return (int)hipGetLastError();
}

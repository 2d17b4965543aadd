// Kernel argument structs shared by the .hip kernels, the native BaB runtime and the bindings.
#pragma once
#include "common.h"

#define FA_MAX_PA 8
#define FA_MAX_RA 8
#define FA_CMAX_PA 8
#define FA_MAX_SPLIT 6      // at most 2^6 children per node and level

struct BoundArgs {
  const float* flat;
  const float* lo;          // [R, n0]  (or node boxes [R/V, n0] when V > 0)
  const float* hi;          // [R, n0]
  const uint8_t* dead_in;   // [R, n_hidden] forced-zero neurons or nullptr
  int R;
  int symbolic;
  int G;                    // box-rows per workgroup
  int stride;               // LDS row stride (floats) of the form buffers
  int wstride;              // LDS row stride of the staged W
  int wfloats;              // LDS floats reserved for the staged W (multiple of 4)
  float* out_lb;            // [R]
  float* out_ub;            // [R]
  float* Lc; float* L0; float* Le;   // [R, n0], [R], [R]  (symbolic)
  float* Uc; float* U0; float* Ue;
  float* layer_lb;          // [R, n_neurons] or nullptr
  float* layer_ub;
  uint8_t* dead_out;        // [R, n_hidden] stable-inactive flags or nullptr
  // node-row expansion: when V > 0, row r is node r / V with its PA dims set to values[r % V]
  int V;
  int npa;
  int pa_idx[FA_MAX_PA];
  const float* values;      // [V, npa]
  // per-partition forced-dead masks (heuristic nets): dead = dead_part[node_part[node]]
  const int* node_part;     // [R / max(V,1)]
  const uint8_t* dead_part; // [P, n_hidden]
  int part_mod;             // > 0: node k uses node_part[k % part_mod] (x rows then x' rows of one
                            //      node list share one part array, no copy)
  // input dims degenerate (lo == hi) in EVERY row: folded into the constant by the
  // register-resident symbolic kernel (PA dims are added automatically when V > 0)
  unsigned long long fold;
  // BaB status filter: rows of nodes whose partition (skip_part[node]) is no longer RUNNING /
  // STOPPING are skipped (nothing written; the split kernel ignores those nodes)
  const int8_t* skip_status;
  const int* skip_part;
  // refine.hip (REFINE + logit, single-PA BaB rows, V > 1): the node's forward logit bounds
  // already exclude every ordered pair of its V rows (out_lb[i] >= 0 or out_ub[j] <= 0 for all
  // i != j -- the certificate's sign shortcut closes it): its rows are not refined
  int skip_signdef;
  // point kernel in the BaB level: point r is the candidate x (r < open_mod) or x' of node
  // r % open_mod; tiles whose 16 points all belong to closed nodes (open == 0, the certificate
  // excluded every pair) are skipped -- the split kernel reads point bounds of open nodes only
  const uint8_t* row_open;
  int open_mod;
  // ReLU-phase rows (relu BaB): [R, n_hidden] int8, -1 = neuron fixed inactive on the row's branch
  // region, +1 = fixed active (identity upper relaxation), 0 = free; rows whose region is proven
  // empty get infeas[r] = 1 (the caller zeroes infeas)
  const int8_t* phase_in;
  uint8_t* infeas;
};

// Inline escalation steps between the first budget and budget2 (fa_settle_kernel): step k has
// budget[k] (increasing, strictly between the two) and the frontier limit open[k] checked at its
// probation level.  n = 0: one step (budget -> budget2, frontier <= max_open).
#define FA_MAX_ESC 4
struct EscSteps {
  int n;
  int budget[FA_MAX_ESC];
  int open[FA_MAX_ESC];
};

struct FwdArgs {
  const float* flat;
  const float* x;          // [B, n0]
  int B;
  const uint8_t* dead;     // [B, n_hidden] or nullptr
  float* out;              // [B]
  int S;
};

// Lattice coordinate ascent of the residual falsifier (engine/falsify.py), one workgroup per
// partition: K starts, +-1 moves on the free (non-protected) dims, every PA assignment.
struct AscentArgs {
  const float* flat;
  const float* lo;          // [P, n0]
  const float* hi;          // [P, n0]
  const float* x0;          // [P, K, n0] start points
  const float* f0;          // [P, K] start margins
  const int* q0;            // [P, K] start pair index
  int P, K, iters;
  int V, npa;
  int pa_idx[FA_MAX_PA];
  const int64_t* values;    // [V, npa]
  int Pp;
  const int64_t* pairs;     // [Pp, 2]
  int nfree;
  int free_idx[64];
  uint8_t* found;           // [P]
  float* wit_x;             // [P, n0]
  float* wit_xp;            // [P, n0]
  int S;
};

// Fused residual falsifier (engine/falsify.py), non-relaxed queries, one workgroup per partition:
// heavy sampling (first strict flip), boundary walk between extreme samples, lattice coordinate
// ascent from the best samples.
struct FalsifyArgs {
  const float* flat;
  const float* lo;          // [P, n0]
  const float* hi;          // [P, n0]
  const int64_t* pids;      // [P]
  int P;
  int n_samples;            // heavy-sampling points per partition
  int n_local;              // the first n_local samples seed the local search
  uint32_t seed;
  int V, npa;
  int pa_idx[FA_MAX_PA];
  const int64_t* values;    // [V, npa]
  int Pp;
  const int64_t* pairs;     // [Pp, 2]
  int walk_k, walk_steps;   // boundary walk: k extreme pairs, bisection steps (0 = off)
  int K, iters;             // local search: starts, coordinate-ascent rounds
  int nfree;
  int free_idx[64];
  uint8_t* found;           // [P]
  float* wit_x;             // [P, n0]
  float* wit_xp;            // [P, n0]
  int8_t* how;              // [P] 0 none, 1 sampling, 2 boundary walk, 3 local search
  // relaxed queries (nra > 0, tau > 0): x' = x with PA value v' and x'_r = x_r + d_r on the RA dims,
  // d_r in [-tau, tau] (unclipped, reference semantics); a sample's offsets come from the hash
  // stream dseed, the local search also moves them; both orientations of every pair count
  int nra;
  int ra_idx[FA_MAX_RA];
  int tau;
  uint32_t dseed;
};

struct SimArgs {
  const float* flat;
  const float* lo;          // [P, n0]
  const float* hi;          // [P, n0]
  const int64_t* pids;      // [P]
  int P;
  int n_samples;
  uint32_t seed;
  int V;                    // PA assignments
  int npa;                  // number of PA dims
  int pa_idx[FA_MAX_PA];
  const int64_t* values;    // [V, npa]
  int Pp;                   // valid ordered pairs
  const int64_t* pairs;     // [Pp, 2]
  int nra;
  int ra_idx[FA_MAX_RA];
  int tau;
  int* counts;              // [P, n_neurons]
  uint8_t* found;           // [P]
  float* wit_x;             // [P, n0]
  float* wit_xp;            // [P, n0]
  float* z0;                // [P, n_samples] logit at PA value 0 (boundary walk) or nullptr
  int* keys;                // [P] first-flip key scratch (INT_MAX-initialised) when split > 1
  int split;                // workgroups per partition (sample tiles strided over them)
  int S;
};

struct CertArgs {
  int Nn, n0, V, Pp, norient;
  const float *Lc, *L0, *Le, *Uc, *U0, *Ue;       // x rows   [Nn*V, n0] / [Nn*V]
  const float *Lcp, *L0p, *Lep, *Ucp, *U0p, *Uep; // x' rows
  const float *olb, *oub, *olbp, *oubp;           // rigorous per-row logit bounds [Nn*V]
  const float *xlo, *xhi, *xplo, *xphi;           // [Nn, n0]
  const int64_t* pairs;                           // [Pp, 2]
  const int64_t* values;                          // [V, npa]
  int npa;
  int pa_idx[FA_CMAX_PA];
  int nra;
  int ra_idx[FA_MAX_RA];
  float tau;
  const uint8_t* shared;                          // [n0]
  float unit;
  float gmarg;                                    // gamma(2*n0+4)
  float* gmin;                                    // [Nn, Q]
  float* tstar;                                   // [Nn, Q]
  // pick outputs
  uint8_t* open;
  float* score;
  int64_t* split_dim;
  float* cand_x;                                  // candidate pair with PA values set, x' clipped
  float* cand_xp;
  int64_t* cand_v;
  int64_t* cand_o;
  float* scores;                                  // [Nn, 2*n0] split scores or nullptr
  uint8_t* leaf;                                  // [Nn] single lattice point (x and x') or nullptr
  // native BaB runtime only: closed nodes write open / score and skip the split scores and the
  // candidate pair (the split kernel reads those for open nodes only), and nodes of partitions
  // that are no longer RUNNING / STOPPING (status[part[n]], the bound kernels' status filter)
  // are closed without evaluating their pairs
  int skip_closed;
  const int8_t* status;
  const int* part;
  // input-split scores from the first layer ("smear", non-relaxed queries): dim i scores
  // width_i * sum over the node's rows of sum_{j unstable in layer 0} |W0[i, j]| instead of the
  // certificate's |coefficient| x width -- a first-layer-dominated net (AC-4 / AC-5 / AC-7: 64-100
  // wide) closes its residue in 30-50 % fewer nodes (tools/diag_open_nodes.py --split smear); the
  // narrow deep nets keep the certificate scores (smear costs them nodes)
  int smear;
  const float* lay_lb;                            // [Nn*V, lay_N] row bounds (layer 0 first)
  const float* lay_ub;
  int lay_N;
  const float* W0T;                               // [n1, 16 or 32] |W0| transposed, zero padded
                                                  // (the row stride is the kernel's NM: n0 <= 16
                                                  // -> 16, else 32)
  int n1;
};

// Level end (fa_settle): per-partition state for the next level, level counters to the host.
// Run by its own launch, or fused into the level's last split launch (P > 0 there).
struct SettleArgs {
  int P;                                  // partitions (0: not fused into this split launch)
  int8_t* status;
  int* lvl_open;
  int* part_open;
  const int* part_nodes;
  int* nodes_start;
  int* prev_start;
  const int* counters_cur;                // this level's (children, candidates)
  int* counters_next;                     // the next level's slot (cleared)
  int* host_counts;                       // pinned host words
  int* pbudget;
  uint8_t* prob;
  int budget2;
  int max_open;
  EscSteps esc;
  int* done;                              // fused: workgroups finished (the last one settles, resets it)
};

// Branch step: close / flag / split the nodes of one sub-batch into the next BFS level.
struct SplitArgs {
  int Nn, n0, relaxed, nra, V, Pp, norient;
  int ra_idx[FA_MAX_RA];
  float tau;
  const float *xlo, *xhi, *xplo, *xphi;   // input nodes [Nn, n0]
  const int* part;                        // [Nn]
  const uint8_t* open;                    // [Nn]
  const uint8_t* leaf;                    // [Nn]
  const float* scores;                    // [Nn, 2*n0]
  const float* cand_x;                    // [Nn, n0]
  const float* cand_xp;
  const float* pe_lb;                     // point-eval bounds: [2*Nn] (x rows then x' rows)
  const float* pe_ub;
  const float *olb, *oub, *olbp, *oubp;   // per-row bounds of the node rows [Nn*V] (leaves)
  const int64_t* pairs;
  const int64_t* values;
  int npa;
  int pa_idx[FA_CMAX_PA];
  const uint8_t* shared;
  int8_t* status;                         // [P]
  int* part_nodes;                        // [P]
  int* part_open;                         // [P] open nodes left unexpanded when the partition
                                          //     stopped (budget / capacity), or nullptr
  int* lvl_open;                          // [P] open inner nodes of this level (reset per level)
  const int* nodes_start;                 // [P] part_nodes at the start of this level
  const int* prev_start;                  // [P] part_nodes at the start of the previous level
                                          //     (nodes_start - prev_start = the partition's nodes
                                          //     in this level; -1 before the first level)
  int budget;
  const int* pbudget;                     // [P] per-partition budget (inline escalation) or nullptr
  uint8_t* prob;                          // [P] probation flags (inline escalation) or nullptr
  int budget2;                            // inline escalation budget
  int m;                                  // largest split-dim count (children = 2^m per node)
  int target;                             // per-partition frontier target of the branching rule
  float *oxlo, *oxhi, *oxplo, *oxphi;     // output pool
  int* opart;
  int* count_out;
  int cap;
  float* cand_buf;                        // [cand_cap, 2*n0+1] candidate records: x, x', then the
                                          //   partition id (int bits), one D2H per level
  int* cand_count;
  int cand_cap;
  SettleArgs settle;                      // fused level end (settle.P > 0: last sub-batch of the level)
};

// BaB solve start (fa_bab_init_kernel): staged host block -> per-partition state + root pool.
struct BabInitArgs {
  int P, n_run, n0;
  const unsigned char* stage;             // device copy of the staged block
  int8_t* status;
  int *nodes, *open_left, *lvl_open, *nodes_start, *prev_start;
  int* part;                              // root pool [n_run]
  float *xlo, *xhi, *xplo, *xphi;         // root pool boxes [n_run, n0] (x' only when relaxed)
  int nra;
  int ra_idx[FA_MAX_RA];
  float tau;
  int* counters;                          // [4]
  int* pbudget;                           // [P] per-partition node budget (inline escalation) or nullptr
  uint8_t* prob;                          // [P] probation flags or nullptr
  int budget;
};

// K1 partition decode (fa_decode_kernel): per input dim, the mixed-radix digit of the id and the
// chunk table slice of its attribute (radix 0 = dim not partitioned: the domain range).
#define FA_DECODE_MAX_DIMS 64
struct DecodeDesc {
  int n0;
  int radix[FA_DECODE_MAX_DIMS];
  long long div[FA_DECODE_MAX_DIMS];      // product of the radices of the attributes after this one
  int chunk_off[FA_DECODE_MAX_DIMS];      // offset of the attribute's chunks in chunk_lo / chunk_hi
  float base_lo[FA_DECODE_MAX_DIMS];
  float base_hi[FA_DECODE_MAX_DIMS];
};

// ReLU-phase backward bounds (relu.hip: fa_crown_phase_kernel, ops/reference.py:crown_phase).
struct CrownPhaseArgs {
  const float* flat;
  const float* lo;          // [R, n0] row boxes (PA dims degenerate)
  const float* hi;
  int R;
  const int8_t* phase;      // [R, n_hidden] or nullptr
  const float* layer_lb;    // [R, n_neurons] forward pre-activation bounds (phase-aware)
  const float* layer_ub;
  const uint8_t* infeas;    // [R] region proven empty by the forward pass, or nullptr
  float* out_lb;            // [R] in: forward logit bounds, out: intersected with the backward ones
  float* out_ub;
  float *Lc, *L0, *Le, *Uc, *U0, *Ue;   // in/out: replaced where the backward input form is tighter
  int* split;               // [R, 2] hidden neuron to split for the lower (0) / upper (1) bound, -1 none
  float* score;             // [R, 2]
  float* low;               // [R, 2] best backward lower bounds of N / -N (or nullptr)
  const int8_t* skip_status;   // rows of partitions no longer RUNNING are skipped (or nullptr)
  const int* skip_part;        // [R]
};

// One BFS level of the ReLU-phase branch-and-bound (relu.hip, csrc/relu_runtime.cpp).  Node n owns
// rows 2n (PA value of its pair's first entry, the copy that must be < 0) and 2n+1 (the copy that
// must be > 0).
struct ReluLevelArgs {
  int Nn, n0, nh;
  int npa;
  int pa_idx[FA_CMAX_PA];
  const int64_t* pairs;     // [Pp, 2] indices into values
  const float* values;      // [V, npa]
  int neg_from;             // > 0: nodes with pair >= neg_from rule out the reverse orientation
                            // N(x, va) > 0 > N(x', vb) (relaxed queries: both orientations in one search;
                            // the pairs table holds every ordered pair twice)
  // input pool
  const int* part;          // [Nn]
  const int* pair;          // [Nn]
  const float* xlo;         // [Nn, n0]
  const float* xhi;
  const int8_t* phase;      // [Nn, 2, nh]
  // rows (written by fa_relu_rows_kernel)
  float* rlo;               // [2 Nn, n0]
  float* rhi;
  int* rpart;               // [2 Nn]
  // per-row bounds (after fa_crown_phase)
  const float* olb;
  const float* oub;
  const uint8_t* infeas;
  const float *Lc, *L0, *Le, *Uc, *U0, *Ue;
  const int* split;         // [2 Nn, 2]
  // certificate outputs
  uint8_t* open;            // [Nn]
  int* choice;              // [Nn] >= 0: row * 65536 + neuron; -1 input split along idim; -2 leaf
  int* idim;                // [Nn]
  float* cpts;              // [2 Nn, n0] candidate points (x with each row's PA values)
  // candidate point bounds
  const float* pe_lb;       // [2 Nn]
  const float* pe_ub;
  // partition state
  int8_t* status;
  int* part_nodes;          // [P] nodes bounded so far (incremented by the rows kernel)
  const int* nodes_start;   // [P] part_nodes at the start of this level (the budget reference)
  int budget;
  // output pool
  int* opart;
  int* opair;
  float* oxlo;
  float* oxhi;
  int8_t* ophase;
  int* count_out;
  int cap;
  float* cand_buf;          // [cand_cap, 2 n0 + 1] x, x', partition id (int bits)
  int* cand_count;
  int cand_cap;
  float unit;
  float gmarg;              // gamma(2 n0 + 4)
  // relaxed queries (|x_r - x'_r| <= tau on the RA dims, x' unclipped): every node also carries x''s
  // box (equal to x's off the RA dims); copy B's row reads it, the certificate concretises the RA
  // dims of the two copies separately (engine/relu_bab.py:certify_pair_relaxed), and a split may
  // halve an x' RA dim (idim >= n0)
  int nra;                  // 0: PA-only query
  int ra_idx[FA_MAX_RA];
  float tau;
  const float* xplo;        // [Nn, n0]
  const float* xphi;
  float* oxplo;             // output pool
  float* oxphi;
};

// beta-CROWN level of the ReLU-phase BaB (csrc/beta.hip, ops/beta.py:level_ref): one wave per node
struct BetaArgs {
  const float* flat;        // network (NetDesc layout)
  const float* wt;          // per layer W_l transposed ([out][in] row-major, at net.w_off[l])
  int R;
  int npa;
  int pa_idx[FA_MAX_PA];
  const float* lo;          // [R, n0] node boxes (PA dims ignored)
  const float* hi;
  const float* va;          // [R, npa] PA values of copy A / copy B
  const float* vb;
  const float* LBA;         // [R, NH] partition pre-activation bounds (unclamped) of copy A / B
  const float* UBA;
  const float* LBB;
  const float* UBB;
  const int8_t* phA;        // [R, NH] phases -1 / 0 / +1
  const int8_t* phB;
  float* par;               // [R, 4, NH] alpha_A, alpha_B, beta_A, beta_B: in = start, out = best
  float* t;                 // [R] in/out
  float* scratch;           // [R, 12, NH] current params, Adam m, Adam v
  int iters;
  float lr_a, lr_b, lr_t, decay;
  int lookahead;            // candidates per score of the filtered branching (0: best gap score)
  int beta_pos;             // project beta >= 0 (1) or keep it free-signed (0)
  int stall;                // 1: when no look-ahead candidate's children beat the node, split the input
  int pgap;                 // > 0: branch by the primal gap mean(h) - relu(mean(z)) of the optimisation's
                            // averaged primal iterates (the verified LP's rule at its optimum); the
                            // iterates' weights: 1 uniform, 2 it + 1, 3 the second half of the steps
  int wpb;                  // waves per workgroup
  int wt_lds;               // 1: transposed weights staged in LDS too
  double* bound;            // [R] rigorous lower bound of t N(x,va) - (1-t) N(x,vb) (+inf: empty region)
  int* split;               // [R] >= 0 neuron (A: j, B: NH + j), -1-d input dim d, -(n0+1) leaf
  float* xstar;             // [R, n0] concretising vertex
  float* binit;             // [R, 2] split multiplier of the (inactive, active) child
  // relaxed queries: copy B reads x' whose RA dims (bit d of ramask) range over [plo, phi] ([R, n0])
  unsigned long long ramask;
  const float* plo;
  const float* phi;
  float* xpstar;            // [R, n0] copy B's vertex (RA dims from x''s box), or nullptr
  float* gtie;              // [R, 2, n0] multipliers of the tie |x_r - x'_r| <= tau (in = start, out =
                            // best), or nullptr (tie dropped)
  float tau;
  const int8_t* osg;        // [R] orientation (+1: N(x,va) < 0 < N(x',vb); -1: the reverse), or nullptr (+1)
  const uint8_t* skip;      // [R] nodes closed before bounding (decided partition, empty region), or nullptr:
                            // bound +inf, no branching
  int ph_stride;            // row stride of phA / phB (0: NH; the native runtime's [R][2][NH] layout: 2 NH)
  int feas;                 // 1: infeasibility pass -- nodes still open (bound < 0) with a fixed phase: the
                            // Lagrangian of the phase constraints alone (objective weight 0, multipliers
                            // in [0, 1]) is optimised; a rigorous value > 0 proves the region empty (bound
                            // := +inf); nothing else is written (scratch must hold [R, 16, NH])
};

// Native beta-CROWN BaB level (csrc/beta_runtime.cpp, kernels csrc/beta_bab.hip): a device-resident
// node pool, double-buffered, structure-of-arrays; node n of the current slice and its children in the
// next pool.  Per node: partition, root tree, orientation, x box, x' box (relaxed), PA values of both
// copies, partition / tightened pre-activation bounds of both copies, phases [2][NH], optimiser
// parameters [4][NH] (alpha_A, alpha_B, beta_A, beta_B), t, tie multipliers [2][n0] (relaxed).
struct BetaPoolArgs {
  int N;                    // nodes in this slice
  int n0, nh, nn;           // input dims, hidden neurons, all neurons (layer-bound row stride)
  int npa;
  int pa_idx[FA_MAX_PA];
  int nra;
  int ra_idx[FA_MAX_RA];
  float tau;
  int leaf;                 // split code of a lattice leaf (-(2 n0 + 1))
  int warm_beta;            // children's split multiplier from binit (else 0)
  int count;                // count kernel: 1 = add the slice's alive nodes to their partitions' counts,
                            // 0 = write the slice's skip flags
  // current slice
  const int* part; const int* tree; const int8_t* osg;
  const float* lo; const float* hi; const float* plo; const float* phi;
  const float* va; const float* vb;
  float* LBA; float* UBA; float* LBB; float* UBB;
  const int8_t* ph; const float* par; const float* t; const float* gt;
  // per partition / per tree
  int8_t* status; int* part_nodes; int budget;
  int* tree_cnt;
  // level work buffers
  uint8_t* skip;            // [N]
  float* rlo; float* rhi; int* rpart;              // [2N, n0] tightening rows (x rows 2n, x' rows 2n+1)
  const float* lay_lb; const float* lay_ub;        // [2N, nn]
  const uint8_t* infeas;                           // [2N]
  const double* bound; const int* split; const float* xstar; const float* xpstar; const float* binit;
  float* cpts;                                     // [2N, n0] candidate points
  const float* pe_lb; const float* pe_ub;          // [2N]
  // next pool
  int* opart; int* otree; int8_t* oosg;
  float* olo; float* ohi; float* oplo; float* ophi; float* ova; float* ovb;
  float* oLBA; float* oUBA; float* oLBB; float* oUBB;
  int8_t* oph; float* opar; float* ot; float* ogt;
  int* count_out; int cap;
  int* nan_count;                    // nodes whose rigorous bound came back NaN (their partition stops)
  int* diag;                         // root level: [0] nodes skipped as not RUNNING, [1] as relaxed-dead
  int root;
  float* cand_buf; int* cand_count; int cand_cap;  // pinned records (x [n0], x' [n0], partition)
};

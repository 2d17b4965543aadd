// Kernel argument structs shared by the .hip kernels and the pybind11 bindings.
#pragma once
#include "common.h"

#define FA_MAX_PA 8
#define FA_MAX_RA 8
#define FA_CMAX_PA 8

struct BoundArgs {
  const float* flat;
  const float* lo;          // [R, n0]
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
};

struct FwdArgs {
  const float* flat;
  const float* x;          // [B, n0]
  int B;
  const uint8_t* dead;     // [B, n_hidden] or nullptr
  float* out;              // [B]
  int S;
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
  int S;
};

struct CertArgs {
  int Nn, n0, V, Pp, norient;
  const float *Lc, *L0, *Le, *Uc, *U0, *Ue;       // x rows   [Nn*V, n0] / [Nn*V]
  const float *Lcp, *L0p, *Lep, *Ucp, *U0p, *Uep; // x' rows
  const float *xlo, *xhi, *xplo, *xphi;           // [Nn, n0]
  const int64_t* pairs;                           // [Pp, 2]
  const int64_t* values;                          // [V, npa]
  int npa;
  int pa_idx[FA_CMAX_PA];
  const uint8_t* shared;                          // [n0]
  float unit;
  float gmarg;                                    // gamma(2*n0+4)
  float* gmin;                                    // [Nn, Q]
  float* tstar;                                   // [Nn, Q]
  // pick outputs
  uint8_t* open;
  float* score;
  int64_t* split_dim;
  float* cand_x;
  float* cand_xp;
  int64_t* cand_v;
  int64_t* cand_o;
};

// Shared host/device layout of the persistent star (parameter-server) ADMM kernel
// (csrc/kernels/star_persistent.hip; reference standared_ADMM.m).
#pragma once
#include "gadmm_chain.h"

struct StarArgs {
  int d, n, n_local, max_iter;   // n: all workers (the hub is worker n - 1)
  int lag, ring, has_monitor, nranks;
  int sys_scope, hub_rank, my_rank;
  int timeline_iters;            // > 0: stamp the first iterations into `timeline` (debug profiling)
  unsigned epoch;                // salts every tag (tag = epoch << 20 | iteration)
  int pad1;
  double rho, obj0, tol;
  long long timeout_ticks;       // s_memrealtime ticks (100 MHz)
  const int* gid;                // [n_local] global worker id of each local workgroup
  const double* Minv;            // [n_local][d][d]: (A + rho I)^-1, the hub's (A + (n-1) rho I)^-1
  const double* A;               // [n_local][d][d]
  const double* b;               // [n_local][d]
  const double* yy;              // [n_local]
  double* theta;                 // [n_local][d] out
  double* lam;                   // [n_local][d] out: worker duals (the hub's row stays 0)
  double* lam_hub;               // [n][d] hub-private copies of the worker duals (hub rank only)
  u32x4* thg;                    // [n][d] this rank's table: worker rows (hub rank) + the hub row
  u32x4* const* peer_thg;        // [nranks] every rank's table (own included)
  u32x4* objg;                   // [ring][n] the monitor rank's objective ring
  unsigned long long* decg;      // [ring] this rank's decision ring
  unsigned long long* const* dec_push;  // [nranks] every rank's decision ring (monitor only)
  double* trace;                 // [max_iter] (monitor rank)
  long long* tstamp;             // [max_iter] decision clock (monitor rank), may be null
  ChainCtl* ctl;
  long long* timeline;           // optional [n_local + 1][timeline_iters][4] s_memrealtime: wait start,
                                 // inputs ready, theta published, objective posted (monitor: decided)
  u32x4* xchk;                   // XCD packing (one GPU): as PersistArgs::xchk / xcd
  int xcd, pad2;
};

/*
 * srbd_oracle.c -- TEST INFRASTRUCTURE ONLY: the CPU oracle for the SRBD-MPC hot path.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this library.
 * The product path (biped_pympc_amd + libsrbd_mpc.so) never calls it.
 *
 * It restates, literally and in FP64, the two reference functions on the hot path:
 *   qp_former                         biped_pympc/casadi/srbd_constraints.py:20-227
 *                                     biped_pympc/casadi/srbd_centroidal_model.py:101-166
 *   sparse_pdipm_multiple_iterations  biped_pympc/casadi/sparse_pdipm_solver.py:357-534
 * CasADi is not installed in this image and the reference ships no fixtures or golden vectors for
 * this path (SURVEY.md sections 4, 8c): PARITY UNPINNED against the reference itself. The oracle is
 * pinned instead by (a) a structural-dependency derivation of the CCS pattern, (b) a second,
 * independent dense restatement (oracle/pdipm_dense.py) agreeing to ~1e-10, and (c) the KKT
 * optimality conditions of the QP at convergence (tests/test_oracle.py).
 *
 * Restatement choices that mirror CasADi:
 *   - jacobian(): forward-mode AD (dual numbers) through the literal RK4 of forward_dynamics.
 *   - b = A z - eq(z), d = G z - ineq(z), f = grad - H z evaluated at the caller's z (x, u inputs).
 *   - ca.ldl / ca.ldl_solve: sparse LDL^T without numeric pivoting after a fill-reducing symmetric
 *     ordering. The checker's ordering is exact minimum degree; CasADi's ldl(A, amd=True) orders by
 *     approximate minimum degree, restated below as a second ordering (amd_order: Amestoy, Davis & Duff
 *     1996 in the form of CSparse's cs_amd, order 1) -- the same maths, the reference's rounding path as
 *     far as the ordering goes (oracle_pdipm_batch_ord; tests/test_oracle.py compares the two).
 *   - if_else(c, a, b) = if_else_zero(c, a) + if_else_zero(!c, b); fmin/fmax are C99 (NaN-ignoring).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define NX 12
#define NU 12
#define F_MAX 500.0
#define LT 0.07
#define LH 0.04
#define DELTA 1e-8
#define BETA 1e-8
#define MAXN 64

/* ------------------------------------------------------------------ dual numbers (AD) --- */
typedef struct { double v, d; } dual;
static inline dual dc(double v) { dual r = {v, 0.0}; return r; }
static inline dual dadd(dual a, dual b) { dual r = {a.v + b.v, a.d + b.d}; return r; }
static inline dual dsub(dual a, dual b) { dual r = {a.v - b.v, a.d - b.d}; return r; }
static inline dual dneg(dual a) { dual r = {-a.v, -a.d}; return r; }
static inline dual dmul(dual a, dual b) { dual r = {a.v * b.v, a.d * b.v + a.v * b.d}; return r; }
static inline dual dkmul(double k, dual a) { dual r = {k * a.v, k * a.d}; return r; }
static inline dual ddivk(dual a, double k) { dual r = {a.v / k, a.d / k}; return r; }

/* casadi.inv of a numeric 3x3 (parameters carry no derivative). */
static void inv3(const double A[3][3], double Ai[3][3]) {
  double c00 = A[1][1] * A[2][2] - A[1][2] * A[2][1];
  double c01 = A[1][2] * A[2][0] - A[1][0] * A[2][2];
  double c02 = A[1][0] * A[2][1] - A[1][1] * A[2][0];
  double det = A[0][0] * c00 + A[0][1] * c01 + A[0][2] * c02;
  Ai[0][0] = c00 / det;
  Ai[1][0] = c01 / det;
  Ai[2][0] = c02 / det;
  Ai[0][1] = (A[0][2] * A[2][1] - A[0][1] * A[2][2]) / det;
  Ai[1][1] = (A[0][0] * A[2][2] - A[0][2] * A[2][0]) / det;
  Ai[2][1] = (A[0][1] * A[2][0] - A[0][0] * A[2][1]) / det;
  Ai[0][2] = (A[0][1] * A[1][2] - A[0][2] * A[1][1]) / det;
  Ai[1][2] = (A[0][2] * A[1][0] - A[0][0] * A[1][2]) / det;
  Ai[2][2] = (A[0][0] * A[1][1] - A[0][1] * A[1][0]) / det;
}

/* SingleRigidBodyDynamics.forward_dynamics, srbd_centroidal_model.py:123-166.
 * params (34): p_body 3 | R 9 (column-major, casadi.reshape) | p_L 3 | p_R 3 | m 1 | I 9 | a_lin 3 | a_ang 3 */
static void forward_dynamics(const dual *st, const dual *in, const double *p, dual *out) {
  double R[3][3], I[3][3], Ii[3][3];
  for (int c = 0; c < 3; ++c)
    for (int r = 0; r < 3; ++r) {
      R[r][c] = p[3 + r + 3 * c];
      I[r][c] = p[19 + r + 3 * c];
    }
  inv3(I, Ii);
  const double mass = p[18];
  const double grav[3] = {0.0, 0.0, -9.81};
  const dual *omega = st + 6, *vel = st + 9;
  const dual *fL = in, *fR = in + 3, *mL = in + 6, *mR = in + 9;
  double rL[3], rR[3];
  for (int k = 0; k < 3; ++k) {
    rL[k] = p[12 + k] - p[k];
    rR[k] = p[15 + k] - p[k];
  }
  /* euler_dot = R @ omega */
  for (int r = 0; r < 3; ++r) {
    dual acc = dc(0.0);
    for (int c = 0; c < 3; ++c) acc = dadd(acc, dkmul(R[r][c], omega[c]));
    out[r] = acc;
  }
  /* com velocity */
  for (int r = 0; r < 3; ++r) out[3 + r] = vel[r];
  /* torque = skew(rL) fL + skew(rR) fR + mL + mR ; skew(v) = [[0,-vz,vy],[vz,0,-vx],[-vy,vx,0]] */
  dual tq[3];
  tq[0] = dadd(dadd(dadd(dsub(dkmul(rL[1], fL[2]), dkmul(rL[2], fL[1])),
                         dsub(dkmul(rR[1], fR[2]), dkmul(rR[2], fR[1]))), mL[0]), mR[0]);
  tq[1] = dadd(dadd(dadd(dsub(dkmul(rL[2], fL[0]), dkmul(rL[0], fL[2])),
                         dsub(dkmul(rR[2], fR[0]), dkmul(rR[0], fR[2]))), mL[1]), mR[1]);
  tq[2] = dadd(dadd(dadd(dsub(dkmul(rL[0], fL[1]), dkmul(rL[1], fL[0])),
                         dsub(dkmul(rR[0], fR[1]), dkmul(rR[1], fR[0]))), mL[2]), mR[2]);
  for (int r = 0; r < 3; ++r) {
    dual acc = dc(0.0);
    for (int c = 0; c < 3; ++c) acc = dadd(acc, dkmul(Ii[r][c], tq[c]));
    out[6 + r] = dadd(acc, dc(p[31 + r]));
  }
  for (int r = 0; r < 3; ++r)
    out[9 + r] = dadd(dadd(ddivk(dadd(fL[r], fR[r]), mass), dc(grav[r])), dc(p[28 + r]));
}

/* rk4_integrator, srbd_centroidal_model.py:101-121 */
static void rk4(const dual *x, const dual *u, const double *p, double dt, dual *xn) {
  dual k1[12], k2[12], k3[12], k4[12], t[12];
  forward_dynamics(x, u, p, k1);
  for (int r = 0; r < 12; ++r) t[r] = dadd(x[r], dkmul(dt / 2, k1[r]));
  forward_dynamics(t, u, p, k2);
  for (int r = 0; r < 12; ++r) t[r] = dadd(x[r], dkmul(dt / 2, k2[r]));
  forward_dynamics(t, u, p, k3);
  for (int r = 0; r < 12; ++r) t[r] = dadd(x[r], dkmul(dt, k3[r]));
  forward_dynamics(t, u, p, k4);
  for (int r = 0; r < 12; ++r) {
    dual s = dadd(dadd(dadd(k1[r], dkmul(2.0, k2[r])), dkmul(2.0, k3[r])), k4[r]);
    xn[r] = dadd(x[r], dkmul(dt / 6, s));
  }
}

/* --------------------------------------------------------------- pattern registry --- */
typedef struct {
  int set;
  int nH, nA, nG;
  int *Hp, *Hi, *Ap, *Ai, *Gp, *Gi;
  /* symbolic LDL of the full KKT (built lazily) */
  int kkt_ready;
  int n, nnzK;
  int *Kp, *Ki;   /* CSC of the permuted-free full symmetric KKT pattern */
  int *Ksrc;      /* per KKT entry: source code (see kkt_fill) */
  struct {        /* per ordering (ORDER_MD exact minimum degree, ORDER_AMD approximate) */
    int ready;
    int *Perm, *Pinv, *Lp, *Parent;
  } sym[2];
} pattern_t;
#define ORDER_MD 0
#define ORDER_AMD 1
static pattern_t g_pat[MAXN + 1];

static int *dupi(const int *a, int n) {
  int *r = (int *)malloc(sizeof(int) * (n > 0 ? n : 1));
  memcpy(r, a, sizeof(int) * n);
  return r;
}

int oracle_set_pattern(int N, const int *Hp, const int *Hi, const int *Ap, const int *Ai,
                       const int *Gp, const int *Gi) {
  if (N < 1 || N > MAXN) return -1;
  pattern_t *P = &g_pat[N];
  if (P->set) return 0; /* immutable once set (thread-safety for the batched calls) */
  const int nz = 24 * N;
  P->nH = Hp[nz];
  P->nA = Ap[nz];
  P->nG = Gp[nz];
  P->Hp = dupi(Hp, nz + 1);
  P->Hi = dupi(Hi, P->nH);
  P->Ap = dupi(Ap, nz + 1);
  P->Ai = dupi(Ai, P->nA);
  P->Gp = dupi(Gp, nz + 1);
  P->Gi = dupi(Gi, P->nG);
  P->set = 1;
  return 0;
}

/* ---------------------------------------------------------------------- qp_former --- */
/* Inputs (srbd_constraints.py:77): x0, x, u, x_ref, dt, m, mu, R_body, I_world, body_pos,
 * left_foot_pos, right_foot_pos, contact_table (N x 2, column-major), Q, R, a_lin, a_ang.
 * Outputs: nonzeros of H, f, A, b, G, d in CCS order. Returns 0, or 1 if a numerically nonzero
 * Jacobian entry falls outside the registered pattern (pattern contract broken). */
int oracle_qp_former(int N, const double *const in[17], double *const out[6]) {
  if (N < 1 || N > MAXN || !g_pat[N].set) return -1;
  const pattern_t *P = &g_pat[N];
  const int nz = 24 * N, neq = 14 * N, nin = 16 * N;
  const double *x0 = in[0], *xv = in[1], *uv = in[2], *xref = in[3];
  const double dt = in[4][0], m = in[5][0], mu = in[6][0];
  const double *ct = in[12], *Q = in[13], *Rw = in[14];
  double params[34];
  /* params = vertcat(p_body, reshape(R_body,9), p_foot1, p_foot2, m, reshape(I_world,9), a_lin, a_ang)
   * (srbd_constraints.py:115) */
  for (int k = 0; k < 3; ++k) params[k] = in[9][k];
  for (int k = 0; k < 9; ++k) params[3 + k] = in[7][k];
  for (int k = 0; k < 3; ++k) params[12 + k] = in[10][k];
  for (int k = 0; k < 3; ++k) params[15 + k] = in[11][k];
  params[18] = m;
  for (int k = 0; k < 9; ++k) params[19 + k] = in[8][k];
  for (int k = 0; k < 3; ++k) params[28 + k] = in[15][k];
  for (int k = 0; k < 3; ++k) params[31 + k] = in[16][k];

  double *A = (double *)calloc((size_t)neq * nz, sizeof(double));
  double *G = (double *)calloc((size_t)nin * nz, sizeof(double));
  double *eq = (double *)calloc(neq, sizeof(double));
  double *iq = (double *)calloc(nin, sizeof(double));
  double *zv = (double *)malloc(sizeof(double) * nz);
  for (int k = 0; k < 12 * N; ++k) {
    zv[k] = xv[k];
    zv[12 * N + k] = uv[k];
  }
#define AD(r, c) A[(size_t)(r) * nz + (c)]
#define GD(r, c) G[(size_t)(r) * nz + (c)]
  /* equality constraints, srbd_constraints.py:118-142 */
  for (int i = 0; i < N; ++i) {
    const double *xi = (i == 0) ? x0 : xv + 12 * (i - 1);
    const double *ui = uv + 12 * i;
    const double *xnext = xv + 12 * i;
    dual xs[12], us[12], xp[12];
    for (int k = 0; k < 12; ++k) { xs[k] = dc(xi[k]); us[k] = dc(ui[k]); }
    rk4(xs, us, params, dt, xp);
    for (int r = 0; r < 12; ++r) {
      eq[12 * i + r] = xnext[r] - xp[r].v;
      AD(12 * i + r, 12 * i + r) = 1.0; /* d x_next / d x_next */
    }
    for (int j = 0; j < 24; ++j) {
      if (j < 12 && i == 0) continue; /* x0 is a parameter, not a decision variable */
      for (int k = 0; k < 12; ++k) { xs[k].d = 0.0; us[k].d = 0.0; }
      if (j < 12) xs[j].d = 1.0; else us[j - 12].d = 1.0;
      rk4(xs, us, params, dt, xp);
      const int col = (j < 12) ? 12 * (i - 1) + j : 12 * N + 12 * i + (j - 12);
      for (int r = 0; r < 12; ++r) AD(12 * i + r, col) = -xp[r].d;
    }
    eq[12 * N + 2 * i] = ui[6];
    eq[12 * N + 2 * i + 1] = ui[9];
    AD(12 * N + 2 * i, 12 * N + 12 * i + 6) = 1.0;
    AD(12 * N + 2 * i + 1, 12 * N + 12 * i + 9) = 1.0;
  }
  /* inequality constraints, srbd_constraints.py:186-227 (duals give the Jacobian) */
  for (int i = 0; i < N; ++i) {
    for (int j = -1; j < 12; ++j) { /* j = -1: value pass; j >= 0: derivative wrt u_i[j] */
      dual u[12];
      for (int k = 0; k < 12; ++k) { u[k] = dc(uv[12 * i + k]); if (k == j) u[k].d = 1.0; }
      const dual dmu = dc(mu);
      dual g[16];
      for (int f = 0; f < 2; ++f) {
        const dual *F = u + 3 * f, *Mm = u + 6 + 3 * f;
        const double c = ct[i + N * f]; /* contact_table[i, f], column-major */
        dual *q = g + 8 * f;
        q[0] = dsub(dneg(F[0]), dmul(dmu, F[2]));
        q[1] = dsub(F[0], dmul(dmu, F[2]));
        q[2] = dsub(dneg(F[1]), dmul(dmu, F[2]));
        q[3] = dsub(F[1], dmul(dmu, F[2]));
        q[4] = dsub(dkmul(-LT, F[2]), Mm[1]);
        q[5] = dadd(dkmul(-LH, F[2]), Mm[1]);
        q[6] = dneg(F[2]);
        q[7] = dsub(F[2], dc(F_MAX * c));
      }
      for (int r = 0; r < 16; ++r) {
        if (j < 0) iq[16 * i + r] = g[r].v;
        else GD(16 * i + r, 12 * N + 12 * i + j) = g[r].d;
      }
    }
  }
  int bad = 0;
  /* gather CCS nonzeros; check the pattern covers every numerically nonzero entry */
  {
    char *mark = (char *)calloc((size_t)neq * nz, 1);
    for (int c = 0; c < nz; ++c)
      for (int p = P->Ap[c]; p < P->Ap[c + 1]; ++p) {
        out[2][p] = AD(P->Ai[p], c);
        mark[(size_t)P->Ai[p] * nz + c] = 1;
      }
    for (size_t e = 0; e < (size_t)neq * nz; ++e)
      if (!mark[e] && A[e] != 0.0) bad = 1;
    free(mark);
    mark = (char *)calloc((size_t)nin * nz, 1);
    for (int c = 0; c < nz; ++c)
      for (int p = P->Gp[c]; p < P->Gp[c + 1]; ++p) {
        out[4][p] = GD(P->Gi[p], c);
        mark[(size_t)P->Gi[p] * nz + c] = 1;
      }
    for (size_t e = 0; e < (size_t)nin * nz; ++e)
      if (!mark[e] && G[e] != 0.0) bad = 1;
    free(mark);
  }
  /* b = A z - eq(z) ; d = G z - ineq(z)   (casadi mtimes: column-ordered accumulation) */
  {
    double *Az = (double *)calloc(neq, sizeof(double));
    for (int c = 0; c < nz; ++c)
      for (int p = P->Ap[c]; p < P->Ap[c + 1]; ++p) Az[P->Ai[p]] += out[2][p] * zv[c];
    for (int r = 0; r < neq; ++r) out[3][r] = Az[r] - eq[r];
    free(Az);
    double *Gz = (double *)calloc(nin, sizeof(double));
    for (int c = 0; c < nz; ++c)
      for (int p = P->Gp[c]; p < P->Gp[c + 1]; ++p) Gz[P->Gi[p]] += out[4][p] * zv[c];
    for (int r = 0; r < nin; ++r) out[5][r] = Gz[r] - iq[r];
    free(Gz);
  }
  /* H = hessian(cost) = diag(Q..., R...); f = grad - H z  (srbd_constraints.py:64-69) */
  for (int c = 0; c < nz; ++c)
    for (int p = P->Hp[c]; p < P->Hp[c + 1]; ++p) {
      const int r = P->Hi[p];
      out[0][p] = (r == c) ? ((c < 12 * N) ? Q[c % 12] : Rw[c % 12]) : 0.0;
    }
  for (int k = 0; k < 12 * N; ++k) {
    const double gx = Q[k % 12] * (xv[k] - xref[k]);
    out[1][k] = gx - Q[k % 12] * xv[k];
    const double gu = Rw[k % 12] * uv[k];
    out[1][12 * N + k] = gu - Rw[k % 12] * uv[k];
  }
  free(A); free(G); free(eq); free(iq); free(zv);
#undef AD
#undef GD
  return bad;
}

/* ------------------------------------------------------------- sparse LDL^T (ca.ldl) --- */
/* Source codes of a KKT entry (value filled per Newton iteration):
 *   code >= 0            : H_val[code]           (+BETA added when the entry is diagonal)
 *   -1 - k  (k < nnzG)   : G_val[k]
 *   ENC_A(k)             : A_val[k]
 *   ENC_W(i)             : 1/s_i * z_i + DELTA   (S^-1 Z + delta I)
 *   ENC_ONE              : +1 (identity blocks)
 *   ENC_MD               : -DELTA
 *   ENC_BETA             : BETA alone (diagonal of x without an H entry) */
#define ENC_BASE_A (-(1 << 24))
#define ENC_BASE_W (-(1 << 26))
#define ENC_ONE (-(1 << 28))
#define ENC_MD (-(1 << 28) - 1)
#define ENC_BETA (-(1 << 28) - 2)

typedef struct { int r, c, src; } trip_t;
static int trip_cmp(const void *a, const void *b) {
  const trip_t *x = (const trip_t *)a, *y = (const trip_t *)b;
  if (x->c != y->c) return x->c - y->c;
  return x->r - y->r;
}

/* exact minimum-degree ordering on a symmetric pattern (bitset elimination graph) */
static void min_degree(int n, const int *Kp, const int *Ki, int *perm) {
  const int W = (n + 63) / 64;
  uint64_t *adj = (uint64_t *)calloc((size_t)n * W, sizeof(uint64_t));
  char *done = (char *)calloc(n, 1);
  for (int c = 0; c < n; ++c)
    for (int p = Kp[c]; p < Kp[c + 1]; ++p) {
      int r = Ki[p];
      if (r != c) {
        adj[(size_t)c * W + r / 64] |= 1ull << (r % 64);
        adj[(size_t)r * W + c / 64] |= 1ull << (c % 64);
      }
    }
  for (int k = 0; k < n; ++k) {
    int best = -1, bestd = 1 << 30;
    for (int v = 0; v < n; ++v) {
      if (done[v]) continue;
      int d = 0;
      for (int w = 0; w < W; ++w) d += __builtin_popcountll(adj[(size_t)v * W + w]);
      if (d < bestd) { bestd = d; best = v; }
    }
    perm[k] = best;
    done[best] = 1;
    uint64_t *nb = adj + (size_t)best * W;
    for (int v = 0; v < n; ++v) { /* neighbours of best become a clique */
      if (!(nb[v / 64] >> (v % 64) & 1)) continue;
      uint64_t *av = adj + (size_t)v * W;
      for (int w = 0; w < W; ++w) av[w] |= nb[w];
      av[v / 64] &= ~(1ull << (v % 64));
      av[best / 64] &= ~(1ull << (best % 64));
    }
    for (int w = 0; w < W; ++w) nb[w] = 0;
  }
  free(adj);
  free(done);
}

/* Approximate minimum degree ordering of a symmetric pattern (the ordering CasADi's ldl(A, amd=True)
 * applies before its LDL^T). Restated from the published algorithm -- Amestoy, Davis & Duff, "An
 * approximate minimum degree ordering algorithm", SIAM J. Matrix Anal. Appl. 17(4), 1996 -- in the form
 * T. A. Davis gives it as cs_amd (Direct Methods for Sparse Linear Systems, SIAM 2006, section 7.1) with
 * order 1 (the pattern of A + A^T without its diagonal): a quotient graph of variables and elements,
 * approximate external degrees |Le \ Lk| from one scan of the element lists, mass elimination,
 * aggressive element absorption, indistinguishable-variable (supervariable) detection by hashing,
 * dense rows (degree > max(16, 10 sqrt n)) ordered last, and the assembly tree postordered. Tie-breaks
 * follow that form: degree lists are LIFO, the pivot is the head of the lowest non-empty list. The
 * quotient graph gets enough elbow room that it is never compacted (compaction moves lists, not their
 * order, so the ordering is the same). Kp / Ki: CSC of a symmetric pattern (diagonal allowed, ignored);
 * perm[k] = the k-th variable eliminated. Returns 0, or -1 on allocation failure. */
#define AMD_FLIP(i) (-(i) - 2)
static int amd_clear(int mark, int lemax, int *w, int n) {
  if (mark < 2 || mark + lemax < 0) {
    for (int k = 0; k < n; ++k)
      if (w[k] != 0) w[k] = 1;
    mark = 2;
  }
  return mark;
}
static int amd_postorder_dfs(int j, int k, int *head, const int *next, int *post, int *stack) {
  int top = 0;
  stack[0] = j;
  while (top >= 0) {
    const int p = stack[top];
    const int i = head[p];
    if (i == -1) {
      top--;
      post[k++] = p;
    } else {
      head[p] = next[i];
      stack[++top] = i;
    }
  }
  return k;
}
static int amd_order(int n, const int *Kp, const int *Ki, int *perm) {
  /* quotient graph storage: the off-diagonal pattern, then room for every element list */
  int cnz = 0;
  for (int c = 0; c < n; ++c)
    for (int q = Kp[c]; q < Kp[c + 1]; ++q) cnz += Ki[q] != c;
  const long cap = (long)cnz + (long)n * (n + 1) + 16;
  int *Cp = (int *)malloc(sizeof(int) * (n + 1)), *Ci = (int *)malloc(sizeof(int) * cap);
  int *W = (int *)malloc(sizeof(int) * 8 * (n + 1)), *P = (int *)malloc(sizeof(int) * (n + 1));
  if (!Cp || !Ci || !W || !P) { free(Cp); free(Ci); free(W); free(P); return -1; }
  for (int c = 0, t = 0; c < n; ++c) {
    Cp[c] = t;
    for (int q = Kp[c]; q < Kp[c + 1]; ++q)
      if (Ki[q] != c) Ci[t++] = Ki[q];
  }
  Cp[n] = cnz;
  int *len = W, *nv = W + (n + 1), *next = W + 2 * (n + 1), *head = W + 3 * (n + 1);
  int *elen = W + 4 * (n + 1), *degree = W + 5 * (n + 1), *w = W + 6 * (n + 1), *hhead = W + 7 * (n + 1);
  int *last = P; /* last[] shares the output array, as the postorder overwrites it at the end */
  int dense = (int)fmax(16.0, 10.0 * sqrt((double)n));
  if (dense > n - 2) dense = n - 2;
  for (int k = 0; k < n; ++k) len[k] = Cp[k + 1] - Cp[k];
  len[n] = 0;
  for (int i = 0; i <= n; ++i) {
    head[i] = last[i] = next[i] = hhead[i] = -1;
    nv[i] = 1;
    w[i] = 1;
    elen[i] = 0;
    degree[i] = len[i];
  }
  int mark = amd_clear(0, 0, w, n), nel = 0, mindeg = 0, lemax = 0;
  elen[n] = -2;
  Cp[n] = -1;
  w[n] = 0;
  for (int i = 0; i < n; ++i) { /* degree lists; empty and dense variables leave at once */
    const int d = degree[i];
    if (d == 0) {
      elen[i] = -2;
      nel++;
      Cp[i] = -1;
      w[i] = 0;
    } else if (d > dense) {
      nv[i] = 0;
      elen[i] = -1;
      nel++;
      Cp[i] = AMD_FLIP(n);
      nv[n]++;
    } else {
      if (head[d] != -1) last[head[d]] = i;
      next[i] = head[d];
      head[d] = i;
    }
  }
  while (nel < n) {
    int k = -1;
    for (; mindeg < n && (k = head[mindeg]) == -1; mindeg++) {
    }
    if (next[k] != -1) last[next[k]] = -1;
    head[mindeg] = next[k];
    const int elenk = elen[k];
    int nvk = nv[k];
    nel += nvk;
    /* the new element Lk: the variables of k's elements and of k's own list */
    int dk = 0;
    nv[k] = -nvk;
    int p = Cp[k];
    const int pk1 = (elenk == 0) ? p : cnz;
    int pk2 = pk1;
    for (int k1 = 1; k1 <= elenk + 1; k1++) {
      int e, pj, ln;
      if (k1 > elenk) {
        e = k;
        pj = p;
        ln = len[k] - elenk;
      } else {
        e = Ci[p++];
        pj = Cp[e];
        ln = len[e];
      }
      for (int k2 = 1; k2 <= ln; k2++) {
        const int i = Ci[pj++];
        const int nvi = nv[i];
        if (nvi <= 0) continue;
        dk += nvi;
        nv[i] = -nvi;
        Ci[pk2++] = i;
        if (next[i] != -1) last[next[i]] = last[i];
        if (last[i] != -1) next[last[i]] = next[i];
        else head[degree[i]] = next[i];
      }
      if (e != k) {
        Cp[e] = AMD_FLIP(k);
        w[e] = 0;
      }
    }
    if (elenk != 0) cnz = pk2;
    degree[k] = dk;
    Cp[k] = pk1;
    len[k] = pk2 - pk1;
    elen[k] = -2;
    /* |Le \ Lk| for every element e adjacent to Lk */
    mark = amd_clear(mark, lemax, w, n);
    for (int pk = pk1; pk < pk2; pk++) {
      const int i = Ci[pk];
      const int eln = elen[i];
      if (eln <= 0) continue;
      const int nvi = -nv[i];
      const int wnvi = mark - nvi;
      for (int q = Cp[i]; q <= Cp[i] + eln - 1; q++) {
        const int e = Ci[q];
        if (w[e] >= mark) w[e] -= nvi;
        else if (w[e] != 0) w[e] = degree[e] + wnvi;
      }
    }
    /* approximate degrees of the variables of Lk; prune their lists; hash them */
    for (int pk = pk1; pk < pk2; pk++) {
      const int i = Ci[pk];
      const int p1 = Cp[i], p2 = p1 + elen[i] - 1;
      int pn = p1, d = 0;
      long h = 0;
      for (int q = p1; q <= p2; q++) {
        const int e = Ci[q];
        if (w[e] != 0) {
          const int dext = w[e] - mark;
          if (dext > 0) {
            d += dext;
            Ci[pn++] = e;
            h += e;
          } else {
            Cp[e] = AMD_FLIP(k); /* aggressive absorption */
            w[e] = 0;
          }
        }
      }
      elen[i] = pn - p1 + 1;
      const int p3 = pn, p4 = p1 + len[i];
      for (int q = p2 + 1; q < p4; q++) {
        const int j = Ci[q];
        const int nvj = nv[j];
        if (nvj <= 0) continue;
        d += nvj;
        Ci[pn++] = j;
        h += j;
      }
      if (d == 0) { /* mass elimination */
        Cp[i] = AMD_FLIP(k);
        const int nvi = -nv[i];
        dk -= nvi;
        nvk += nvi;
        nel += nvi;
        nv[i] = 0;
        elen[i] = -1;
      } else {
        if (d < degree[i]) degree[i] = d;
        Ci[pn] = Ci[p3];
        Ci[p3] = Ci[p1];
        Ci[p1] = k;
        len[i] = pn - p1 + 1;
        const int hb = (int)((h < 0 ? -h : h) % n);
        next[i] = hhead[hb];
        hhead[hb] = i;
        last[i] = hb;
      }
    }
    degree[k] = dk;
    if (dk > lemax) lemax = dk;
    mark = amd_clear(mark + lemax, lemax, w, n);
    /* supervariables: variables of Lk with identical lists (one hash bucket at a time) */
    for (int pk = pk1; pk < pk2; pk++) {
      int i = Ci[pk];
      if (nv[i] >= 0) continue;
      const int hb = last[i];
      i = hhead[hb];
      hhead[hb] = -1;
      for (; i != -1 && next[i] != -1; i = next[i], mark++) {
        const int ln = len[i], eln = elen[i];
        for (int q = Cp[i] + 1; q <= Cp[i] + ln - 1; q++) w[Ci[q]] = mark;
        int jlast = i;
        for (int j = next[i]; j != -1;) {
          int ok = (len[j] == ln) && (elen[j] == eln);
          for (int q = Cp[j] + 1; ok && q <= Cp[j] + ln - 1; q++)
            if (w[Ci[q]] != mark) ok = 0;
          if (ok) {
            Cp[j] = AMD_FLIP(i);
            nv[i] += nv[j];
            nv[j] = 0;
            elen[j] = -1;
            j = next[j];
            next[jlast] = j;
          } else {
            jlast = j;
            j = next[j];
          }
        }
      }
    }
    /* back into the degree lists with their external degrees */
    int pw = pk1;
    for (int pk = pk1; pk < pk2; pk++) {
      const int i = Ci[pk];
      const int nvi = -nv[i];
      if (nvi <= 0) continue;
      nv[i] = nvi;
      int d = degree[i] + dk - nvi;
      if (d > n - nel - nvi) d = n - nel - nvi;
      if (head[d] != -1) last[head[d]] = i;
      next[i] = head[d];
      last[i] = -1;
      head[d] = i;
      if (d < mindeg) mindeg = d;
      degree[i] = d;
      Ci[pw++] = i;
    }
    nv[k] = nvk;
    if ((len[k] = pw - pk1) == 0) {
      Cp[k] = -1;
      w[k] = 0;
    }
    if (elenk != 0) cnz = pw;
    if ((long)cnz + (long)n >= cap) { free(Cp); free(Ci); free(W); free(P); return -1; }
  }
  /* postorder the assembly tree: absorbed variables and elements under their parents */
  for (int i = 0; i < n; ++i) Cp[i] = AMD_FLIP(Cp[i]);
  for (int j = 0; j <= n; ++j) head[j] = -1;
  for (int j = n; j >= 0; j--) {
    if (nv[j] > 0) continue;
    next[j] = head[Cp[j]];
    head[Cp[j]] = j;
  }
  for (int e = n; e >= 0; e--) {
    if (nv[e] <= 0) continue;
    if (Cp[e] != -1) {
      next[e] = head[Cp[e]];
      head[Cp[e]] = e;
    }
  }
  for (int k = 0, i = 0; i <= n; i++)
    if (Cp[i] == -1) k = amd_postorder_dfs(i, k, head, next, P, w);
  memcpy(perm, P, sizeof(int) * n); /* P[n] is the dense-row root n */
  free(Cp); free(Ci); free(W); free(P);
  return 0;
}

/* amd_order of an arbitrary symmetric CSC pattern (tests/test_oracle.py pins it on small graphs) */
int oracle_amd_order(int n, const int *Kp, const int *Ki, int *perm) { return n < 1 ? -1 : amd_order(n, Kp, Ki, perm); }

/* the full KKT pattern of sparse_pdipm_solver.py:412-439 (shared by both orderings) */
static int build_kkt_pattern(int N) {
  pattern_t *P = &g_pat[N];
  if (P->kkt_ready) return 0;
  const int nz = 24 * N, m = 16 * N, p = 14 * N, n = nz + 2 * m + p;
  const int cap = 2 * (P->nH + P->nA + P->nG) + 4 * n + 16;
  trip_t *T = (trip_t *)malloc(sizeof(trip_t) * cap);
  int nt = 0;
  /* top-left: Q + beta I (union pattern), sparse_pdipm_solver.py:419 */
  char *hasdiag = (char *)calloc(nz, 1);
  for (int c = 0; c < nz; ++c)
    for (int q = P->Hp[c]; q < P->Hp[c + 1]; ++q) {
      T[nt++] = (trip_t){P->Hi[q], c, q};
      if (P->Hi[q] == c) hasdiag[c] = 1;
    }
  for (int c = 0; c < nz; ++c)
    if (!hasdiag[c]) T[nt++] = (trip_t){c, c, ENC_BETA};
  free(hasdiag);
  /* G^T (rows 0..nz, cols nz+m..) and G (rows nz+m.., cols 0..nz), :422,:431 */
  for (int c = 0; c < nz; ++c)
    for (int q = P->Gp[c]; q < P->Gp[c + 1]; ++q) {
      T[nt++] = (trip_t){nz + m + P->Gi[q], c, -1 - q};
      T[nt++] = (trip_t){c, nz + m + P->Gi[q], -1 - q};
    }
  /* A^T and A, :424,:434 */
  for (int c = 0; c < nz; ++c)
    for (int q = P->Ap[c]; q < P->Ap[c + 1]; ++q) {
      T[nt++] = (trip_t){nz + 2 * m + P->Ai[q], c, ENC_BASE_A - q};
      T[nt++] = (trip_t){c, nz + 2 * m + P->Ai[q], ENC_BASE_A - q};
    }
  for (int i = 0; i < m; ++i) {
    T[nt++] = (trip_t){nz + i, nz + i, ENC_BASE_W - i};        /* S^-1 Z + delta I, :427 */
    T[nt++] = (trip_t){nz + i, nz + m + i, ENC_ONE};           /* I, :428 */
    T[nt++] = (trip_t){nz + m + i, nz + i, ENC_ONE};           /* I, :432 */
    T[nt++] = (trip_t){nz + m + i, nz + m + i, ENC_MD};        /* -delta I, :437 */
  }
  for (int i = 0; i < p; ++i) T[nt++] = (trip_t){nz + 2 * m + i, nz + 2 * m + i, ENC_MD}; /* :439 */
  qsort(T, nt, sizeof(trip_t), trip_cmp);
  P->n = n;
  P->nnzK = nt;
  P->Kp = (int *)calloc(n + 1, sizeof(int));
  P->Ki = (int *)malloc(sizeof(int) * nt);
  P->Ksrc = (int *)malloc(sizeof(int) * nt);
  for (int e = 0; e < nt; ++e) {
    P->Kp[T[e].c + 1]++;
    P->Ki[e] = T[e].r;
    P->Ksrc[e] = T[e].src;
  }
  for (int c = 0; c < n; ++c) P->Kp[c + 1] += P->Kp[c];
  free(T);
  P->kkt_ready = 1;
  return 0;
}

/* ordering `order` of the KKT and ldl_symbolic (elimination tree + column counts) on the permuted
 * matrix. Built once per (N, order), before any batch loop (the batched entry points are parallel). */
static int build_kkt_symbolic_ord(int N, int order) {
  if (order != ORDER_MD && order != ORDER_AMD) return -1;
  if (build_kkt_pattern(N)) return -1;
  pattern_t *P = &g_pat[N];
  if (P->sym[order].ready) return 0;
  const int n = P->n;
  int *Perm = (int *)malloc(sizeof(int) * n), *Pinv = (int *)malloc(sizeof(int) * n);
  if (order == ORDER_MD) min_degree(n, P->Kp, P->Ki, Perm);
  else if (amd_order(n, P->Kp, P->Ki, Perm)) { free(Perm); free(Pinv); return -1; }
  for (int k = 0; k < n; ++k) Pinv[k] = -1;
  for (int k = 0; k < n; ++k) {
    if (Perm[k] < 0 || Perm[k] >= n || Pinv[Perm[k]] != -1) { free(Perm); free(Pinv); return -1; }
    Pinv[Perm[k]] = k;
  }
  int *Lp = (int *)malloc(sizeof(int) * (n + 1)), *Parent = (int *)malloc(sizeof(int) * n);
  int *Lnz = (int *)malloc(sizeof(int) * n), *Flag = (int *)malloc(sizeof(int) * n);
  for (int k = 0; k < n; ++k) {
    Parent[k] = -1;
    Flag[k] = k;
    Lnz[k] = 0;
    const int kk = Perm[k];
    for (int q = P->Kp[kk]; q < P->Kp[kk + 1]; ++q) {
      int i = Pinv[P->Ki[q]];
      if (i < k)
        for (; Flag[i] != k; i = Parent[i]) {
          if (Parent[i] == -1) Parent[i] = k;
          Lnz[i]++;
          Flag[i] = k;
        }
    }
  }
  Lp[0] = 0;
  for (int k = 0; k < n; ++k) Lp[k + 1] = Lp[k] + Lnz[k];
  free(Lnz);
  free(Flag);
  P->sym[order].Perm = Perm;
  P->sym[order].Pinv = Pinv;
  P->sym[order].Lp = Lp;
  P->sym[order].Parent = Parent;
  P->sym[order].ready = 1;
  return 0;
}
static int build_kkt_symbolic(int N) { return build_kkt_symbolic_ord(N, ORDER_MD); }

int oracle_prepare_solver(int N) {
  if (N < 1 || N > MAXN || !g_pat[N].set) return -1;
  return build_kkt_symbolic(N);
}

/* the KKT size, its nonzeros and those of L under ordering `order` (0 exact minimum degree, 1 AMD) */
int oracle_kkt_stats_ord(int N, int order, int *n, int *nnzK, int *nnzL) {
  if (N < 1 || N > MAXN || !g_pat[N].set || build_kkt_symbolic_ord(N, order)) return -1;
  *n = g_pat[N].n;
  *nnzK = g_pat[N].nnzK;
  *nnzL = g_pat[N].sym[order].Lp[g_pat[N].n];
  return 0;
}
int oracle_kkt_stats(int N, int *n, int *nnzK, int *nnzL) { return oracle_kkt_stats_ord(N, ORDER_MD, n, nnzK, nnzL); }

/* the elimination order itself (perm[k] = KKT row eliminated k-th); returns n or -1 */
int oracle_kkt_order(int N, int order, int *perm) {
  if (N < 1 || N > MAXN || !g_pat[N].set || build_kkt_symbolic_ord(N, order)) return -1;
  memcpy(perm, g_pat[N].sym[order].Perm, sizeof(int) * g_pat[N].n);
  return g_pat[N].n;
}

/* column pointers of L (nnz per column = Lp[j+1] - Lp[j]) for flop accounting */
int oracle_kkt_lp(int N, int *Lp_out) {
  if (oracle_prepare_solver(N)) return -1;
  memcpy(Lp_out, g_pat[N].sym[ORDER_MD].Lp, sizeof(int) * (g_pat[N].n + 1));
  return g_pat[N].n;
}

typedef struct {
  double *Kx, *Lx, *D, *Y;
  int *Li, *Lnz, *Pattern, *Flag;
} ldl_work;

/* ldl_numeric (up-looking LDL^T, no pivoting) */
typedef struct {
  const int *Perm, *Pinv, *Lp, *Parent;
} sym_ref;
static int ldl_numeric(const pattern_t *P, sym_ref S, ldl_work *w) {
  const int n = P->n;
  int fail = 0;  /* first zero pivot (1-based); the factorisation still runs to the end, so every column
                    of L has its pattern and ldl_solve stays in bounds (the values are then inf / NaN) */
  for (int k = 0; k < n; ++k) {
    w->Y[k] = 0.0;
    int top = n;
    w->Flag[k] = k;
    w->Lnz[k] = 0;
    const int kk = S.Perm[k];
    for (int q = P->Kp[kk]; q < P->Kp[kk + 1]; ++q) {
      int i = S.Pinv[P->Ki[q]];
      if (i <= k) {
        w->Y[i] += w->Kx[q];
        int len;
        for (len = 0; w->Flag[i] != k; i = S.Parent[i]) {
          w->Pattern[len++] = i;
          w->Flag[i] = k;
        }
        while (len > 0) w->Pattern[--top] = w->Pattern[--len];
      }
    }
    w->D[k] = w->Y[k];
    w->Y[k] = 0.0;
    for (; top < n; top++) {
      const int i = w->Pattern[top];
      const double yi = w->Y[i];
      w->Y[i] = 0.0;
      const int p2 = S.Lp[i] + w->Lnz[i];
      int q;
      for (q = S.Lp[i]; q < p2; q++) w->Y[w->Li[q]] -= w->Lx[q] * yi;
      const double l_ki = yi / w->D[i];
      w->D[k] -= l_ki * yi;
      w->Li[q] = k;
      w->Lx[q] = l_ki;
      w->Lnz[i]++;
    }
    if (w->D[k] == 0.0 && !fail) fail = k + 1;
  }
  return fail;
}

/* ldl_solve: x = P^T L^-T D^-1 L^-1 P b  (b overwritten with the solution) */
static void ldl_solve(const pattern_t *P, sym_ref S, const ldl_work *w, double *b, double *tmp) {
  const int n = P->n;
  for (int k = 0; k < n; ++k) tmp[k] = b[S.Perm[k]];
  for (int j = 0; j < n; ++j)
    for (int q = S.Lp[j]; q < S.Lp[j + 1]; ++q) tmp[w->Li[q]] -= w->Lx[q] * tmp[j];
  for (int j = 0; j < n; ++j) tmp[j] /= w->D[j];
  for (int j = n - 1; j >= 0; --j)
    for (int q = S.Lp[j]; q < S.Lp[j + 1]; ++q) tmp[j] -= w->Lx[q] * tmp[w->Li[q]];
  for (int k = 0; k < n; ++k) b[S.Perm[k]] = tmp[k];
}

/* sparse mat-vec helpers with CasADi's column-ordered accumulation */
static void spmv(int ncol, const int *Cp, const int *Ci, const double *v, const double *x, double *y) {
  for (int c = 0; c < ncol; ++c)
    for (int q = Cp[c]; q < Cp[c + 1]; ++q) y[Ci[q]] += v[q] * x[c];
}
static void spmv_t(int ncol, const int *Cp, const int *Ci, const double *v, const double *x, double *y) {
  for (int c = 0; c < ncol; ++c) {
    double acc = 0.0;
    for (int q = Cp[c]; q < Cp[c + 1]; ++q) acc += v[q] * x[Ci[q]];
    y[c] += acc;
  }
}

static double step_length(int m, const double *v, const double *dv) {
  /* fmax(fmin(1, 0.99 * mmin_i if_else(dv_i < 0, -v_i/dv_i, 1)), 1e-12), :460-467 */
  double mn = INFINITY;
  for (int i = 0; i < m; ++i) {
    const int c = dv[i] < 0.0;
    const double a = -v[i] / dv[i];
    const double cand = (c ? a : 0.0) + (!c ? 1.0 : 0.0);
    mn = fmin(mn, cand);
  }
  return fmax(fmin(1.0, 0.99 * mn), 1e-12);
}

/* Per-problem status word (not a reference output; the build's failure-detection hook, SURVEY.md 5,
 * computed here with the same definition as the HIP kernels so tests can compare them):
 * bit 0 -- a non-finite value in the returned x, s, z, y or mu; bit 1 -- a combined-direction step
 * length (primal or dual) at its 1e-12 floor (sparse_pdipm_solver.py:501-502) in the last iteration.
 * (Bit 2, "solved by the general fallback", exists only on the GPU.) Bit 3 is the oracle's own: its
 * sparse LDL^T met a zero pivot in some iteration (the batch entry points then return 0 and report
 * the failure only here), so a test comparing GPU and oracle words sees an oracle that failed. */
#define ORACLE_STATUS_LDL_FAIL 8
static int nonfinite(const double *v, int n) {
  for (int i = 0; i < n; ++i)
    if (!isfinite(v[i])) return 1;
  return 0;
}

/* sparse_pdipm_multiple_iterations, sparse_pdipm_solver.py:357-534.
 * in : Q_val, G_val, A_val, f, h, b, x, s, z, y        out: x, s, z, y, residuals(4), mu(1)
 * status: NULL, or the status word above. */
static int pdipm_ord(int N, int n_iter, const double *const in[10], double *const out[6], int *status, int order) {
  if (N < 1 || N > MAXN || !g_pat[N].set || n_iter < 1) return -1;
  if (build_kkt_symbolic_ord(N, order)) return -1;
  const pattern_t *P = &g_pat[N];
  const sym_ref S = {P->sym[order].Perm, P->sym[order].Pinv, P->sym[order].Lp, P->sym[order].Parent};
  const int nz = 24 * N, m = 16 * N, p = 14 * N, n = P->n;
  const double *Hv = in[0], *Gv = in[1], *Av = in[2], *f = in[3], *h = in[4], *b = in[5];
  double *x = (double *)malloc(sizeof(double) * nz), *s = (double *)malloc(sizeof(double) * m);
  double *z = (double *)malloc(sizeof(double) * m), *y = (double *)malloc(sizeof(double) * p);
  memcpy(x, in[6], sizeof(double) * nz);
  memcpy(s, in[7], sizeof(double) * m);
  memcpy(z, in[8], sizeof(double) * m);
  memcpy(y, in[9], sizeof(double) * p);
  ldl_work w;
  const int nnzL = S.Lp[n];
  w.Kx = (double *)malloc(sizeof(double) * P->nnzK);
  w.Lx = (double *)malloc(sizeof(double) * (nnzL > 0 ? nnzL : 1));
  w.Li = (int *)malloc(sizeof(int) * (nnzL > 0 ? nnzL : 1));
  w.D = (double *)malloc(sizeof(double) * n);
  w.Y = (double *)malloc(sizeof(double) * n);
  w.Lnz = (int *)malloc(sizeof(int) * n);
  w.Pattern = (int *)malloc(sizeof(int) * n);
  w.Flag = (int *)malloc(sizeof(int) * n);
  double *rx = (double *)malloc(sizeof(double) * nz), *rs = (double *)malloc(sizeof(double) * m);
  double *re = (double *)malloc(sizeof(double) * p), *tmp = (double *)malloc(sizeof(double) * n);
  double *sa = (double *)malloc(sizeof(double) * n), *sc = (double *)malloc(sizeof(double) * n);
  double *Gx = (double *)malloc(sizeof(double) * m), *sinv = (double *)malloc(sizeof(double) * m);
  double res[4] = {0, 0, 0, 0}, mu_new = 0.0;
  int rc = 0;
  for (int it = 0; it < n_iter; ++it) {
    /* residuals, :392-402 */
    memset(rx, 0, sizeof(double) * nz);
    spmv(nz, P->Hp, P->Hi, Hv, x, rx);                 /* Qx */
    for (int k = 0; k < nz; ++k) rx[k] += f[k];          /* + f */
    spmv_t(nz, P->Gp, P->Gi, Gv, z, rx);                 /* + G^T z */
    spmv_t(nz, P->Ap, P->Ai, Av, y, rx);                 /* + A^T y */
    memset(re, 0, sizeof(double) * p);
    spmv(nz, P->Ap, P->Ai, Av, x, re);
    for (int k = 0; k < p; ++k) re[k] -= b[k];
    memset(Gx, 0, sizeof(double) * m);
    spmv(nz, P->Gp, P->Gi, Gv, x, Gx);
    for (int k = 0; k < m; ++k) rs[k] = Gx[k] + s[k] - h[k];
    double sz = 0.0;
    for (int k = 0; k < m; ++k) sz += s[k] * z[k];
    const double mu = sz / m;
    /* KKT values, :412-439 */
    for (int k = 0; k < m; ++k) sinv[k] = 1.0 / s[k];
    for (int e = 0; e < P->nnzK; ++e) {
      const int src = P->Ksrc[e];
      double v;
      if (src >= 0) v = Hv[src]; /* beta is added to its diagonal entries below */
      else if (src == ENC_ONE) v = 1.0;
      else if (src == ENC_MD) v = -DELTA;
      else if (src == ENC_BETA) v = BETA;
      else if (src <= ENC_BASE_W && src > ENC_BASE_W - (1 << 25)) { const int i = ENC_BASE_W - src; v = sinv[i] * z[i] + DELTA; }
      else if (src <= ENC_BASE_A && src > ENC_BASE_A - (1 << 23)) v = Av[ENC_BASE_A - src];
      else v = Gv[-1 - src];
      w.Kx[e] = v;
    }
    /* + beta on the diagonal of the H block where H has an entry */
    for (int c = 0; c < nz; ++c)
      for (int q = P->Kp[c]; q < P->Kp[c + 1]; ++q)
        if (P->Ki[q] == c && P->Ksrc[q] >= 0) w.Kx[q] += BETA;
    const int fail = ldl_numeric(P, S, &w);
    if (fail) rc = 2;
    /* affine rhs = [-rx; -(S^-1 (s o z)); -rs; -re] */
    for (int k = 0; k < nz; ++k) sa[k] = -rx[k];
    for (int k = 0; k < m; ++k) sa[nz + k] = -(sinv[k] * (s[k] * z[k]));
    for (int k = 0; k < m; ++k) sa[nz + m + k] = -rs[k];
    for (int k = 0; k < p; ++k) sa[nz + 2 * m + k] = -re[k];
    ldl_solve(P, S, &w, sa, tmp);
    const double *dxa = sa, *dsa = sa + nz, *dza = sa + nz + m;
    const double ap = step_length(m, s, dsa), ad = step_length(m, z, dza);
    double sza = 0.0;
    for (int k = 0; k < m; ++k) sza += (s[k] + ap * dsa[k]) * (z[k] + ad * dza[k]);
    const double mu_aff = sza / m;
    const double sigma = pow(mu_aff / mu, 3.0);
    /* corrector rhs = [0; -S^-1 (s o z + ds_a o dz_a - sigma mu e); 0; 0] */
    for (int k = 0; k < n; ++k) sc[k] = 0.0;
    for (int k = 0; k < m; ++k) {
      const double rcc = s[k] * z[k] + dsa[k] * dza[k] - sigma * mu * 1.0;
      sc[nz + k] = -(sinv[k] * rcc);
    }
    ldl_solve(P, S, &w, sc, tmp);
    (void)dxa;
    for (int k = 0; k < n; ++k) sc[k] = sa[k] + sc[k]; /* combined direction */
    const double *dx = sc, *ds = sc + nz, *dz = sc + nz + m, *dy = sc + nz + 2 * m;
    const double apc = step_length(m, s, ds), adc = step_length(m, z, dz);
    const int floor_hit = apc <= 1e-12 || adc <= 1e-12;
    if (status && it == n_iter - 1) *status = floor_hit ? 2 : 0;
    for (int k = 0; k < nz; ++k) x[k] = x[k] + apc * dx[k];
    for (int k = 0; k < m; ++k) s[k] = fmax(s[k] + apc * ds[k], 1e-8);
    for (int k = 0; k < m; ++k) z[k] = fmax(fmax(z[k] + adc * dz[k], 1e-8), 1e-8);
    for (int k = 0; k < p; ++k) y[k] = y[k] + adc * dy[k];
    double szn = 0.0;
    for (int k = 0; k < m; ++k) szn += s[k] * z[k];
    mu_new = szn / m;
    double nx_ = 0, ns_ = 0, ne_ = 0;
    for (int k = 0; k < nz; ++k) nx_ += rx[k] * rx[k];
    for (int k = 0; k < m; ++k) ns_ += rs[k] * rs[k];
    for (int k = 0; k < p; ++k) ne_ += re[k] * re[k];
    res[0] = sqrt(nx_);
    res[1] = sqrt(ns_);
    res[2] = sqrt(ne_);
    res[3] = mu_new;
  }
  memcpy(out[0], x, sizeof(double) * nz);
  memcpy(out[1], s, sizeof(double) * m);
  memcpy(out[2], z, sizeof(double) * m);
  memcpy(out[3], y, sizeof(double) * p);
  memcpy(out[4], res, sizeof(double) * 4);
  out[5][0] = mu_new;
  if (status && (nonfinite(x, nz) || nonfinite(s, m) || nonfinite(z, m) || nonfinite(y, p) || !isfinite(mu_new)))
    *status |= 1;
  if (status && rc) *status |= ORACLE_STATUS_LDL_FAIL;
  free(x); free(s); free(z); free(y);
  free(w.Kx); free(w.Lx); free(w.Li); free(w.D); free(w.Y); free(w.Lnz); free(w.Pattern); free(w.Flag);
  free(rx); free(rs); free(re); free(tmp); free(sa); free(sc); free(Gx); free(sinv);
  return rc;
}

int oracle_pdipm_st(int N, int n_iter, const double *const in[10], double *const out[6], int *status) {
  return pdipm_ord(N, n_iter, in, out, status, ORDER_MD);
}

int oracle_pdipm(int N, int n_iter, const double *const in[10], double *const out[6]) {
  return oracle_pdipm_st(N, n_iter, in, out, NULL);
}

/* -------------------------------------------------------------- batched wrappers --- */
/* Row-major (B, nnz) arrays per tensor, as CusADi lays out its batched buffers
 * (CusadiFunction.py:71-76). OpenMP over envs mirrors evaluate_parallel_cpu.cpp:79. */
static const int FORMER_NNZ_FIXED[17] = {12, -12, -12, -12, 1, 1, 1, 9, 9, 3, 3, 3, -2, 12, 12, 3, 3};

static int former_nnz(int N, int i) { int v = FORMER_NNZ_FIXED[i]; return v > 0 ? v : -v * N; }

int oracle_qp_former_batch(int N, int B, const double *const in[17], double *const out[6], int nthreads) {
  if (N < 1 || N > MAXN || !g_pat[N].set) return -1;
  const pattern_t *P = &g_pat[N];
  const int onnz[6] = {P->nH, 24 * N, P->nA, 14 * N, P->nG, 16 * N};
  int bad = 0;
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 4) reduction(| : bad)
#endif
  for (int e = 0; e < B; ++e) {
    const double *pi[17];
    double *po[6];
    for (int i = 0; i < 17; ++i) pi[i] = in[i] + (size_t)e * former_nnz(N, i);
    for (int i = 0; i < 6; ++i) po[i] = out[i] + (size_t)e * onnz[i];
    bad |= oracle_qp_former(N, pi, po) != 0;
  }
  return bad;
}

/* oracle_pdipm_batch under elimination order `order` (0: the checker's exact minimum degree, 1: AMD,
 * the ordering of CasADi's ldl) */
int oracle_pdipm_batch_ord(int N, int n_iter, int B, const double *const in[10], double *const out[6],
                           int nthreads, int *status, int order) {
  if (N < 1 || N > MAXN || !g_pat[N].set) return -1;
  if (build_kkt_symbolic_ord(N, order)) return -1;
  const pattern_t *P = &g_pat[N];
  const int innz[10] = {P->nH, P->nG, P->nA, 24 * N, 16 * N, 14 * N, 24 * N, 16 * N, 16 * N, 14 * N};
  const int onnz[6] = {24 * N, 16 * N, 16 * N, 14 * N, 4, 1};
  int bad = 0;
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 1) reduction(| : bad)
#endif
  for (int e = 0; e < B; ++e) {
    const double *pi[10];
    double *po[6];
    for (int i = 0; i < 10; ++i) pi[i] = in[i] + (size_t)e * innz[i];
    for (int i = 0; i < 6; ++i) po[i] = out[i] + (size_t)e * onnz[i];
    bad |= pdipm_ord(N, n_iter, pi, po, status ? status + e : NULL, order) != 0;
  }
  return status ? 0 : bad;
}

int oracle_pdipm_batch(int N, int n_iter, int B, const double *const in[10], double *const out[6], int nthreads,
                       int *status) {
  return oracle_pdipm_batch_ord(N, n_iter, B, in, out, nthreads, status, ORDER_MD);
}

/* The GPU caller's full MPC step per env (mpc_controller_cusadi.py:99-169): qp_former, then
 * x = 0, s = max(d - G.0, 1), z = 1, y = y0, then n_iter Newton iterations. */
int oracle_mpc_solve_batch(int N, int n_iter, double y0, int B, const double *const in[17],
                           double *const out[6], int nthreads, int *status) {
  if (N < 1 || N > MAXN || !g_pat[N].set) return -1;
  if (build_kkt_symbolic(N)) return -1;
  const pattern_t *P = &g_pat[N];
  const int onnz[6] = {24 * N, 16 * N, 16 * N, 14 * N, 4, 1};
  int bad = 0;
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 1) reduction(| : bad)
#endif
  for (int e = 0; e < B; ++e) {
    const double *pi[17];
    for (int i = 0; i < 17; ++i) pi[i] = in[i] + (size_t)e * former_nnz(N, i);
    const int nz = 24 * N, m = 16 * N, p = 14 * N;
    double *H = (double *)malloc(sizeof(double) * P->nH), *f = (double *)malloc(sizeof(double) * nz);
    double *A = (double *)malloc(sizeof(double) * P->nA), *b = (double *)malloc(sizeof(double) * p);
    double *G = (double *)malloc(sizeof(double) * P->nG), *d = (double *)malloc(sizeof(double) * m);
    double *qo[6] = {H, f, A, b, G, d};
    bad |= oracle_qp_former(N, pi, qo) != 0;
    double *x = (double *)calloc(nz, sizeof(double)), *s = (double *)malloc(sizeof(double) * m);
    double *z = (double *)malloc(sizeof(double) * m), *y = (double *)malloc(sizeof(double) * p);
    /* s = max(d - G @ 0, 1): G @ 0 is exactly 0 for finite G */
    double *Gx = (double *)calloc(m, sizeof(double));
    spmv(nz, P->Gp, P->Gi, G, x, Gx);
    for (int k = 0; k < m; ++k) { s[k] = fmax(d[k] - Gx[k], 1.0); z[k] = 1.0; }
    for (int k = 0; k < p; ++k) y[k] = y0;
    const double *si[10] = {H, G, A, f, d, b, x, s, z, y};
    double *so[6];
    for (int i = 0; i < 6; ++i) so[i] = out[i] + (size_t)e * onnz[i];
    bad |= oracle_pdipm_st(N, n_iter, si, so, status ? status + e : NULL) != 0;
    free(H); free(f); free(A); free(b); free(G); free(d); free(x); free(s); free(z); free(y); free(Gx);
  }
  return status ? 0 : bad;
}

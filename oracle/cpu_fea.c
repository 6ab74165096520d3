/*
 * cpu_fea.c — CPU restatement of one FEA load step, TEST/BASELINE INFRASTRUCTURE ONLY.
 *
 * Used by tests/ (checker) and by bench.py's cpu_baseline leg (the "host PETSc
 * CG" of BASELINE.md §3).  Never linked into libmfea.so.
 *
 * Restates, in plain C + OpenMP:
 *   element_stiffness_6x6            src/fea_petsc.cpp:88-140
 *   assembly (ADD_VALUES semantics)  src/fea_petsc.cpp:229-263, into a CSR pattern
 *                                    built once per mesh (MatSetValue w/o
 *                                    preallocation is the reference's cost model;
 *                                    the pattern phase is timed separately)
 *   Dirichlet elimination + reg      src/fea_solver.py:112-125 (free-block system,
 *                                    +reg on the K_ff diagonal only)
 *   KSPCG + PCJACOBI                 PETSc 3.24.1 src/ksp/ksp/impls/cg/cg.c (not
 *                                    vendored): standard Hestenes–Stiefel PCG, x0 = 0;
 *                                    stopping on the unpreconditioned residual
 *                                    ‖r‖ ≤ rtol·‖b‖ (SURVEY §8d metric, SciPy cg)
 *   reactions + stress               src/fea_petsc.cpp:360-406
 *
 * Build: gcc -O3 -march=native -fopenmp -shared -fPIC cpu_fea.c -o libcpu_fea.so -lm
 */
#include <math.h>
#include <omp.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
  int64_t N, E, nf;      /* nodes, elements, free nodes                         */
  int64_t *node_free;    /* orig node -> free index (or -1)                      */
  int64_t *row_ptr;      /* CSR over 3N DOFs (orig order), node-block pattern    */
  int32_t *col;
  int64_t *slot;         /* per element: 4 block positions (11,12,21,22) into val */
  double *val;
  const double *xyz;
  const int64_t *e2n;
  uint8_t *code;         /* 0 free, 1 top, 2 bottom (bottom overrides top)       */
  int64_t n_top;
  const int64_t *top;
} cpu_mesh;

static double EA_, EI12_, EMOD_;

/* src/fea_petsc.cpp:88-140 (identical arithmetic to the Python bulk form) */
static void element_S(const double *p1, const double *p2, double S[3][3]) {
  double vx = p2[0] - p1[0], vy = p2[1] - p1[1], vz = p2[2] - p1[2];
  double L = sqrt(vx * vx + vy * vy + vz * vz);
  if (L < 1e-12) L = 1e-12;
  double n[3] = {vx / L, vy / L, vz / L};
  double kax = EA_ / L, kb = EI12_ / (L * L * L);
  for (int a = 0; a < 3; ++a)
    for (int b = 0; b < 3; ++b) {
      double tt = n[a] * n[b];
      S[a][b] = tt * kax + ((a == b ? 1.0 : 0.0) - tt) * kb;
    }
}

static int cmp_i64(const void *a, const void *b) {
  int64_t x = *(const int64_t *)a, y = *(const int64_t *)b;
  return x < y ? -1 : x > y;
}

void cpu_set_material(double E, double A, double I) {
  EA_ = E * A;
  EI12_ = (12.0 * E) * I;
  EMOD_ = E;
}

/* Pattern: one CSR row per DOF, a 3-wide column block per neighbour node. */
cpu_mesh *cpu_mesh_create(int64_t N, const double *xyz, int64_t E, const int64_t *e2n,
                          int64_t n_top, const int64_t *top, int64_t n_bot, const int64_t *bot) {
  cpu_mesh *m = (cpu_mesh *)calloc(1, sizeof(cpu_mesh));
  m->N = N; m->E = E; m->xyz = xyz; m->e2n = e2n; m->n_top = n_top; m->top = top;
  m->code = (uint8_t *)calloc(N ? N : 1, 1);
  for (int64_t i = 0; i < n_top; ++i) m->code[top[i]] = 1;
  for (int64_t i = 0; i < n_bot; ++i) m->code[bot[i]] = 2;
  m->node_free = (int64_t *)malloc(sizeof(int64_t) * (N ? N : 1));
  m->nf = 0;
  for (int64_t n = 0; n < N; ++n) m->node_free[n] = m->code[n] ? -1 : m->nf++;
  /* neighbour lists */
  int64_t *deg = (int64_t *)calloc(N + 1, sizeof(int64_t));
  for (int64_t e = 0; e < E; ++e) { deg[e2n[2 * e]]++; deg[e2n[2 * e + 1]]++; }
  int64_t *nptr = (int64_t *)calloc(N + 1, sizeof(int64_t));
  for (int64_t n = 0; n < N; ++n) nptr[n + 1] = nptr[n] + deg[n] + 1;
  int64_t *nb = (int64_t *)malloc(sizeof(int64_t) * (nptr[N] ? nptr[N] : 1));
  int64_t *fill = (int64_t *)malloc(sizeof(int64_t) * (N ? N : 1));
  for (int64_t n = 0; n < N; ++n) { fill[n] = nptr[n]; nb[fill[n]++] = n; }
  for (int64_t e = 0; e < E; ++e) {
    int64_t a = e2n[2 * e], b = e2n[2 * e + 1];
    nb[fill[a]++] = b; nb[fill[b]++] = a;
  }
  int64_t *ulen = (int64_t *)malloc(sizeof(int64_t) * (N ? N : 1));
  for (int64_t n = 0; n < N; ++n) {
    qsort(nb + nptr[n], nptr[n + 1] - nptr[n], sizeof(int64_t), cmp_i64);
    int64_t w = nptr[n];
    for (int64_t k = nptr[n]; k < nptr[n + 1]; ++k)
      if (k == nptr[n] || nb[k] != nb[k - 1]) nb[w++] = nb[k];
    ulen[n] = w - nptr[n];
  }
  m->row_ptr = (int64_t *)calloc(3 * N + 1, sizeof(int64_t));
  for (int64_t n = 0; n < N; ++n)
    for (int a = 0; a < 3; ++a) m->row_ptr[3 * n + a + 1] = m->row_ptr[3 * n + a] + 3 * ulen[n];
  int64_t nnz = m->row_ptr[3 * N];
  m->col = (int32_t *)malloc(sizeof(int32_t) * (nnz ? nnz : 1));
  m->val = (double *)calloc(nnz ? nnz : 1, sizeof(double));
  for (int64_t n = 0; n < N; ++n)
    for (int a = 0; a < 3; ++a) {
      int64_t p = m->row_ptr[3 * n + a];
      for (int64_t k = 0; k < ulen[n]; ++k)
        for (int b = 0; b < 3; ++b) m->col[p++] = (int32_t)(3 * nb[nptr[n] + k] + b);
    }
  /* per element the position of blocks (a,a), (a,b), (b,a), (b,b) in row 3a / 3b */
  m->slot = (int64_t *)malloc(sizeof(int64_t) * 4 * (E ? E : 1));
  for (int64_t e = 0; e < E; ++e) {
    int64_t na = e2n[2 * e], nbn = e2n[2 * e + 1];
    int64_t ends[2] = {na, nbn};
    for (int i = 0; i < 2; ++i)
      for (int j = 0; j < 2; ++j) {
        int64_t r = ends[i], c = ends[j];
        int64_t lo = nptr[r], hi = nptr[r] + ulen[r];
        while (lo < hi) { int64_t mid = (lo + hi) / 2; if (nb[mid] < c) lo = mid + 1; else hi = mid; }
        m->slot[4 * e + 2 * i + j] = m->row_ptr[3 * r] + 3 * (lo - nptr[r]);
      }
  }
  free(deg); free(nptr); free(nb); free(fill); free(ulen);
  return m;
}

void cpu_mesh_destroy(cpu_mesh *m) {
  if (!m) return;
  free(m->code); free(m->node_free); free(m->row_ptr); free(m->col); free(m->val); free(m->slot);
  free(m);
}

/* ADD_VALUES assembly in element order (serial: preserves the reference's order) */
static void assemble(cpu_mesh *m, const uint8_t *active) {
  memset(m->val, 0, sizeof(double) * m->row_ptr[3 * m->N]);
  for (int64_t e = 0; e < m->E; ++e) {
    if (!active[e]) continue;
    int64_t a = m->e2n[2 * e], b = m->e2n[2 * e + 1];
    double S[3][3];
    element_S(m->xyz + 3 * a, m->xyz + 3 * b, S);
    for (int i = 0; i < 2; ++i)
      for (int j = 0; j < 2; ++j) {
        double sg = (i == j) ? 1.0 : -1.0;
        int64_t p0 = m->slot[4 * e + 2 * i + j];
        int64_t r0 = 3 * (i ? b : a);
        for (int ra = 0; ra < 3; ++ra) {
          int64_t off = m->row_ptr[r0 + ra] - m->row_ptr[r0];
          for (int cb = 0; cb < 3; ++cb) m->val[p0 + off + cb] += sg * S[ra][cb];
        }
      }
  }
}

static double now_s(void) { return omp_get_wtime(); }

/*
 * One load step.  active is updated in place (elements failing this step are
 * cleared).  Returns PCG iterations (>=0) or -1 on max_it.
 * times[4] = assemble, rhs, pcg, post seconds.
 */
int cpu_fea_step(cpu_mesh *m, uint8_t *active, double dy_top, double dy_bot, double rtol,
                 int max_it, double reg, double max_strain, int nthreads, double *U,
                 double *stress, double *total_force, double *relres, double *times) {
  if (nthreads > 0) omp_set_num_threads(nthreads);
  const int64_t N = m->N, nf = m->nf, n = 3 * nf;
  double t0 = now_s();
  assemble(m, active);
  double t1 = now_s();
  /* free-DOF system: reuse the full CSR rows of free nodes, skipping known columns */
  double *x = (double *)calloc(n ? n : 1, sizeof(double)), *r = (double *)malloc(sizeof(double) * (n ? n : 1));
  double *p = (double *)malloc(sizeof(double) * (n ? n : 1)), *q = (double *)malloc(sizeof(double) * (n ? n : 1));
  double *dinv = (double *)malloc(sizeof(double) * (n ? n : 1));
  int64_t *frow = (int64_t *)malloc(sizeof(int64_t) * (nf ? nf : 1));
  for (int64_t nd = 0; nd < N; ++nd) if (m->node_free[nd] >= 0) frow[m->node_free[nd]] = nd;
  double bb = 0.0;
#pragma omp parallel for reduction(+ : bb) schedule(static)
  for (int64_t i = 0; i < n; ++i) {
    int64_t row = 3 * frow[i / 3] + i % 3;
    double kx = 0.0, d = 0.0;
    for (int64_t t = m->row_ptr[row]; t < m->row_ptr[row + 1]; ++t) {
      int64_t c = m->col[t], cn = c / 3;
      if (m->code[cn]) { if (c % 3 == 1) kx += m->val[t] * (m->code[cn] == 2 ? dy_bot : dy_top); }
      else if (c == row) d = m->val[t];
    }
    r[i] = 0.0 - kx;
    dinv[i] = 1.0 / (d + reg);
    p[i] = dinv[i] * r[i];
    bb += r[i] * r[i];
  }
  double rho = 0.0;
#pragma omp parallel for reduction(+ : rho) schedule(static)
  for (int64_t i = 0; i < n; ++i) rho += r[i] * p[i];
  double t2 = now_s();
  const double tol2 = rtol * rtol * bb;
  double rr = bb;
  int it = 0;
  while (rr > tol2 && it < max_it) {
    double pq = 0.0;
#pragma omp parallel for reduction(+ : pq) schedule(static)
    for (int64_t i = 0; i < n; ++i) {
      int64_t row = 3 * frow[i / 3] + i % 3;
      double y = 0.0;
      for (int64_t t = m->row_ptr[row]; t < m->row_ptr[row + 1]; ++t) {
        int64_t c = m->col[t], cf = m->node_free[c / 3];
        if (cf >= 0) y += m->val[t] * p[3 * cf + c % 3];
      }
      y += reg * p[i];
      q[i] = y;
      pq += p[i] * y;
    }
    double alpha = rho / pq, rz = 0.0;
    rr = 0.0;
#pragma omp parallel for reduction(+ : rz, rr) schedule(static)
    for (int64_t i = 0; i < n; ++i) {
      x[i] += alpha * p[i];
      r[i] -= alpha * q[i];
      rz += r[i] * dinv[i] * r[i];
      rr += r[i] * r[i];
    }
    double beta = rz / rho;
    rho = rz;
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) p[i] = dinv[i] * r[i] + beta * p[i];
    ++it;
  }
  double t3 = now_s();
  for (int64_t nd = 0; nd < N; ++nd) {
    int64_t f = m->node_free[nd];
    for (int a = 0; a < 3; ++a)
      U[3 * nd + a] = f >= 0 ? x[3 * f + a] : (a == 1 ? (m->code[nd] == 2 ? dy_bot : dy_top) : 0.0);
  }
  double F = 0.0;
  for (int64_t k = 0; k < m->n_top; ++k) {
    int64_t row = 3 * m->top[k] + 1;
    for (int64_t t = m->row_ptr[row]; t < m->row_ptr[row + 1]; ++t) F += m->val[t] * U[m->col[t]];
  }
#pragma omp parallel for schedule(static)
  for (int64_t e = 0; e < m->E; ++e) {
    if (!active[e]) { stress[e] = 0.0; continue; }
    int64_t a = m->e2n[2 * e], b = m->e2n[2 * e + 1];
    double v[3], du[3];
    for (int c = 0; c < 3; ++c) { v[c] = m->xyz[3 * b + c] - m->xyz[3 * a + c]; du[c] = U[3 * b + c] - U[3 * a + c]; }
    double L = sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
    double strain = fma(v[2] / L, du[2], fma(v[1] / L, du[1], (v[0] / L) * du[0])) / L;
    stress[e] = EMOD_ * strain;
    if (fabs(strain) > max_strain) active[e] = 0;
  }
  double t4 = now_s();
  *total_force = F;
  *relres = bb > 0 ? sqrt(rr / bb) : 0.0;
  if (times) { times[0] = t1 - t0; times[1] = t2 - t1; times[2] = t3 - t2; times[3] = t4 - t3; }
  free(x); free(r); free(p); free(q); free(dinv); free(frow);
  return (rr > tol2) ? -1 : it;
}

/* Axial strain exactly as src/fea_solver.py:263-270 computes it: L =
 * np.linalg.norm(v) = sqrt(v·v), n = v/L (no clamp), ε = np.dot(n, u2−u1)/L,
 * where NumPy's length-3 dot is BLAS ddot, an FMA chain
 * (x0·y0 → fma(x1,y1,·) → fma(x2,y2,·)). */
void cpu_strain(int64_t E, const int64_t *e2n, const double *xyz, const double *U, double *out) {
  for (int64_t e = 0; e < E; ++e) {
    int64_t a = e2n[2 * e], b = e2n[2 * e + 1];
    double v0 = xyz[3 * b] - xyz[3 * a], v1 = xyz[3 * b + 1] - xyz[3 * a + 1],
           v2 = xyz[3 * b + 2] - xyz[3 * a + 2];
    /* np.linalg.norm of a 1-D vector is sqrt(x.dot(x)): ddot again (py:266) */
    double L = sqrt(fma(v2, v2, fma(v1, v1, v0 * v0)));
    double n0 = v0 / L, n1 = v1 / L, n2 = v2 / L;
    double d0 = U[3 * b] - U[3 * a], d1 = U[3 * b + 1] - U[3 * a + 1], d2 = U[3 * b + 2] - U[3 * a + 2];
    out[e] = fma(n2, d2, fma(n1, d1, n0 * d0)) / L;
  }
}

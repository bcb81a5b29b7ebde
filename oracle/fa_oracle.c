/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C CPU restatement of the reference's element-stiffness assembly path
 * (SalzmanA/fem-libraries, mechanic2d).  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load this library, and only as the checker or as
 * the timed CPU baseline.  The product path (fem-libraries_amd/) never links it.
 *
 * Parity status: UNPINNED against reference outputs — the reference ships no
 * assembly fixtures and neither FEniCSx 0.8.0 nor MFEM 4.7.0 can be built or imported
 * in this container.  What pins it instead (tests/test_oracle.py):
 *   - glibc srand(6575)/rand() material table, exactly the reference's algorithm
 *     (FEniCSx/mechanic2d/asym_elasto_damage_model.cc:533-545);
 *   - SymPy exact integration of element matrices (independent CAS);
 *   - rigid-body null space, symmetry, partition of unity;
 *   - the damage-law tangent against a SymPy second derivative of the reference
 *     potential psi (FEniCSx/mechanic2d/asym_ufl.py:37-51, MFEM/.../asym_elasto_damage_model.cc:100-155).
 *
 * What is restated, with the reference anchor of each piece:
 *   ora_nodes / ora_tabulate     basix 0.8 Lagrange element (3rd-party; elements chosen at
 *                                FEniCSx/mechanic2d/asym_ufl.py:11-13): nodal basis by Vandermonde
 *                                inversion over monomials, basix sub-entity node ordering,
 *                                GLL-warped 1-D points for tensor degree >= 3.
 *   ora_quadrature               basix default rule (3rd-party): Xiao-Gimbutas for low-degree
 *                                simplices, Gauss-Jacobi (Gauss-Legendre) tensor rules with
 *                                (m+2)/2 points per direction.
 *   ora_elasticity_cell          MFEM damIntegrator::AssembleElementGrad, USE_B branch, linear
 *                                "hook" (MFEM/mechanic2d/asym_elasto_damage_model.cc:684-704,
 *                                :873-887): elmat += w * B * hook * B^T, generalised to 3-D Voigt.
 *   ora_damage_hook              the hand-written tangent of the same integrator
 *                                (MFEM/mechanic2d/asym_elasto_damage_model.cc:735-872).
 *   ora_damage_stress            asym_stress, non-AD (MFEM/mechanic2d/asym_elasto_damage_model.cc:207-329).
 *   ora_assemble_matrix          dolfinx 0.8 fem::assemble_matrix + set_diagonal as called from
 *                                setJ (FEniCSx/mechanic2d/asym_elasto_damage_model.cc:847-862):
 *                                zero A_e, kernel, zero bc rows/cols, ADD into the global matrix,
 *                                then INSERT `diag` on bc diagonal entries.
 *   ora_sparsity                 dolfinx fem::create_sparsity_pattern (3rd-party, called through
 *                                create_matrix at asym_elasto_damage_model.cc:688): all node pairs of
 *                                every cell.
 *
 * Cell-type codes mirror dolfinx::mesh::CellType: triangle 3, quadrilateral 4,
 * tetrahedron -4, hexahedron 8.  Dof layout is dolfinx-blocked: dof = node * bs + comp.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define ORA_TRI 3
#define ORA_QUAD 4
#define ORA_TET (-4)
#define ORA_HEX 8

#define ORA_MAXN 64  /* max nodes per cell (Q3 hex) */
#define ORA_MAXQ 256 /* max quadrature points */

static int tdim_of(int ct) { return (ct == ORA_TRI || ct == ORA_QUAD) ? 2 : 3; }
static int simplex(int ct) { return ct == ORA_TRI || ct == ORA_TET; }

int ora_num_nodes(int ct, int p) {
  switch (ct) {
    case ORA_TRI: return (p + 1) * (p + 2) / 2;
    case ORA_TET: return (p + 1) * (p + 2) * (p + 3) / 6;
    case ORA_QUAD: return (p + 1) * (p + 1);
    case ORA_HEX: return (p + 1) * (p + 1) * (p + 1);
  }
  return -1;
}

/* ---------------------------------------------------------------- reference cells (basix) */
static const double TRI_V[3][3] = {{0, 0, 0}, {1, 0, 0}, {0, 1, 0}};
static const int TRI_E[3][2] = {{1, 2}, {0, 2}, {0, 1}};
static const double TET_V[4][3] = {{0, 0, 0}, {1, 0, 0}, {0, 1, 0}, {0, 0, 1}};
static const int TET_E[6][2] = {{2, 3}, {1, 3}, {1, 2}, {0, 3}, {0, 2}, {0, 1}};
static const double QUAD_V[4][3] = {{0, 0, 0}, {1, 0, 0}, {0, 1, 0}, {1, 1, 0}};
static const int QUAD_E[4][2] = {{0, 1}, {0, 2}, {1, 3}, {2, 3}};
static const double HEX_V[8][3] = {{0, 0, 0}, {1, 0, 0}, {0, 1, 0}, {1, 1, 0},
                                   {0, 0, 1}, {1, 0, 1}, {0, 1, 1}, {1, 1, 1}};
static const int HEX_E[12][2] = {{0, 1}, {0, 2}, {0, 4}, {1, 3}, {1, 5}, {2, 3},
                                 {2, 6}, {3, 7}, {4, 5}, {4, 6}, {5, 7}, {6, 7}};
/* quad faces of the hex: (v0, v1, v2) spanning the face as v0 + s(v1-v0) + t(v2-v0) */
static const int HEX_F[6][3] = {{0, 1, 2}, {0, 1, 4}, {0, 2, 4}, {1, 3, 5}, {2, 3, 6}, {4, 5, 6}};

/* interior 1-D lattice parameters for degree p: equispaced, or GLL (= basix gll_warped in 1-D)
 * for tensor cells at p >= 3. Returns count p-1. */
static int interior_params(int ct, int p, double* r) {
  if (p < 2) return 0;
  if (!simplex(ct) && p == 3) {
    r[0] = 0.5 * (1.0 - 1.0 / sqrt(5.0));
    r[1] = 0.5 * (1.0 + 1.0 / sqrt(5.0));
    return 2;
  }
  for (int k = 1; k < p; ++k) r[k - 1] = (double)k / p;
  return p - 1;
}

/* Reference node coordinates in basix ordering: vertices, edges, faces, interior.
 * Supported: simplex p in {1,2}; tensor p in {1,2,3}. Returns node count or -1. */
int ora_nodes(int ct, int p, double* X /* [n][3] */) {
  int n = 0, td = tdim_of(ct);
  double r[8];
  int ni = interior_params(ct, p, r);
  if (simplex(ct) && p > 2) return -1;
  if (!simplex(ct) && p > 3) return -1;
  const double(*V)[3];
  const int(*E)[2];
  int nv, ne;
  switch (ct) {
    case ORA_TRI: V = TRI_V; E = TRI_E; nv = 3; ne = 3; break;
    case ORA_TET: V = TET_V; E = TET_E; nv = 4; ne = 6; break;
    case ORA_QUAD: V = QUAD_V; E = QUAD_E; nv = 4; ne = 4; break;
    case ORA_HEX: V = HEX_V; E = HEX_E; nv = 8; ne = 12; break;
    default: return -1;
  }
  for (int v = 0; v < nv; ++v) {
    for (int d = 0; d < 3; ++d) X[3 * n + d] = V[v][d];
    ++n;
  }
  for (int e = 0; e < ne; ++e)
    for (int k = 0; k < ni; ++k) {
      for (int d = 0; d < 3; ++d) X[3 * n + d] = V[E[e][0]][d] + r[k] * (V[E[e][1]][d] - V[E[e][0]][d]);
      ++n;
    }
  if (ct == ORA_QUAD) { /* cell interior: first parameter slowest */
    for (int i = 0; i < ni; ++i)
      for (int j = 0; j < ni; ++j) {
        X[3 * n + 0] = r[i]; X[3 * n + 1] = r[j]; X[3 * n + 2] = 0; ++n;
      }
  }
  if (ct == ORA_HEX) {
    for (int f = 0; f < 6; ++f)
      for (int i = 0; i < ni; ++i)
        for (int j = 0; j < ni; ++j) {
          const double* a = V[HEX_F[f][0]];
          const double* b = V[HEX_F[f][1]];
          const double* c = V[HEX_F[f][2]];
          for (int d = 0; d < 3; ++d) X[3 * n + d] = a[d] + r[i] * (b[d] - a[d]) + r[j] * (c[d] - a[d]);
          ++n;
        }
    for (int i = 0; i < ni; ++i)
      for (int j = 0; j < ni; ++j)
        for (int k = 0; k < ni; ++k) {
          X[3 * n + 0] = r[i]; X[3 * n + 1] = r[j]; X[3 * n + 2] = r[k]; ++n;
        }
  }
  (void)td;
  return n;
}

/* ---------------------------------------------------------------- polynomial space */
static int monomials(int ct, int p, int (*ex)[3]) {
  int m = 0, td = tdim_of(ct);
  for (int k = 0; k <= (td == 3 ? p : 0); ++k)
    for (int j = 0; j <= p; ++j)
      for (int i = 0; i <= p; ++i) {
        if (simplex(ct) && i + j + k > p) continue;
        ex[m][0] = i; ex[m][1] = j; ex[m][2] = k; ++m;
      }
  return m;
}

/* Shifted Legendre polynomial L_e(t) = P_e(2t-1) and its derivative (three-term recurrence).
 * Products of these span the same spaces as monomials but give a well-conditioned
 * Vandermonde matrix at degree 3 on hexahedra. */
static void legendre01(int e, double t, double* v, double* dv) {
  double z = 2.0 * t - 1.0;
  double p0 = 1.0, p1 = z, d0 = 0.0, d1 = 1.0;
  if (e == 0) { *v = 1.0; *dv = 0.0; return; }
  for (int k = 2; k <= e; ++k) {
    double p2 = ((2.0 * k - 1.0) * z * p1 - (k - 1.0) * p0) / k;
    double d2 = ((2.0 * k - 1.0) * (p1 + z * d1) - (k - 1.0) * d0) / k;
    p0 = p1; p1 = p2; d0 = d1; d1 = d2;
  }
  *v = p1;
  *dv = 2.0 * d1;
}

/* value and gradient of L_a(x) L_b(y) L_c(z) */
static void mono_eval(const int* e, const double* x, double* v, double* g) {
  double px, py, pz, dx, dy, dz;
  legendre01(e[0], x[0], &px, &dx);
  legendre01(e[1], x[1], &py, &dy);
  legendre01(e[2], x[2], &pz, &dz);
  *v = px * py * pz;
  g[0] = dx * py * pz;
  g[1] = px * dy * pz;
  g[2] = px * py * dz;
}

/* in-place Gauss-Jordan inverse with partial pivoting, n x n row-major. 0 on success. */
static int invert(int n, double* A) {
  double* Inv = (double*)calloc((size_t)n * n, sizeof(double));
  for (int i = 0; i < n; ++i) Inv[i * n + i] = 1.0;
  for (int c = 0; c < n; ++c) {
    int piv = c;
    for (int r = c + 1; r < n; ++r)
      if (fabs(A[r * n + c]) > fabs(A[piv * n + c])) piv = r;
    if (fabs(A[piv * n + c]) < 1e-300) { free(Inv); return -1; }
    if (piv != c)
      for (int k = 0; k < n; ++k) {
        double t = A[c * n + k]; A[c * n + k] = A[piv * n + k]; A[piv * n + k] = t;
        t = Inv[c * n + k]; Inv[c * n + k] = Inv[piv * n + k]; Inv[piv * n + k] = t;
      }
    double d = 1.0 / A[c * n + c];
    for (int k = 0; k < n; ++k) { A[c * n + k] *= d; Inv[c * n + k] *= d; }
    for (int r = 0; r < n; ++r) {
      if (r == c) continue;
      double f = A[r * n + c];
      if (f == 0.0) continue;
      for (int k = 0; k < n; ++k) { A[r * n + k] -= f * A[c * n + k]; Inv[r * n + k] -= f * Inv[c * n + k]; }
    }
  }
  memcpy(A, Inv, sizeof(double) * n * n);
  free(Inv);
  return 0;
}

/* Tabulate the nodal Lagrange basis (values [np][nn], reference gradients [np][nn][tdim]).
 * Returns nn or -1. */
int ora_tabulate(int ct, int p, int np, const double* pts /* [np][tdim] */, double* vals, double* grads) {
  double X[ORA_MAXN * 3];
  int ex[ORA_MAXN][3];
  int td = tdim_of(ct);
  int nn = ora_nodes(ct, p, X);
  if (nn < 0) return -1;
  int nm = monomials(ct, p, ex);
  if (nm != nn) return -1;
  double* Vm = (double*)malloc(sizeof(double) * nn * nn);
  for (int i = 0; i < nn; ++i)
    for (int m = 0; m < nm; ++m) {
      double g[3];
      mono_eval(ex[m], &X[3 * i], &Vm[i * nn + m], g);
    }
  if (invert(nn, Vm)) { free(Vm); return -1; }
  /* C = V^{-1}: phi_n(x) = sum_m C[m][n] mono_m(x) */
  for (int q = 0; q < np; ++q) {
    double x[3] = {0, 0, 0};
    for (int d = 0; d < td; ++d) x[d] = pts[q * td + d];
    double mv[ORA_MAXN], mg[ORA_MAXN][3];
    for (int m = 0; m < nm; ++m) mono_eval(ex[m], x, &mv[m], mg[m]);
    for (int n = 0; n < nn; ++n) {
      double v = 0, g[3] = {0, 0, 0};
      for (int m = 0; m < nm; ++m) {
        double c = Vm[m * nn + n];
        v += c * mv[m];
        for (int d = 0; d < 3; ++d) g[d] += c * mg[m][d];
      }
      if (vals) vals[q * nn + n] = v;
      if (grads)
        for (int d = 0; d < td; ++d) grads[(q * nn + n) * td + d] = g[d];
    }
  }
  free(Vm);
  return nn;
}

/* ---------------------------------------------------------------- quadrature */
/* Gauss-Legendre on [0,1] by Newton iteration on P_n. */
static void gauss_legendre01(int n, double* x, double* w) {
  for (int i = 0; i < n; ++i) {
    double z = cos(M_PI * (i + 0.75) / (n + 0.5)), pp = 0;
    for (int it = 0; it < 100; ++it) {
      double p0 = 1.0, p1 = z;
      for (int k = 2; k <= n; ++k) {
        double p2 = ((2.0 * k - 1.0) * z * p1 - (k - 1.0) * p0) / k;
        p0 = p1; p1 = p2;
      }
      if (n == 1) { p1 = z; p0 = 1.0; }
      pp = n * (z * p1 - p0) / (z * z - 1.0);
      double dz = p1 / pp;
      z -= dz;
      if (fabs(dz) < 1e-16) break;
    }
    {
      double p0 = 1.0, p1 = z;
      for (int k = 2; k <= n; ++k) {
        double p2 = ((2.0 * k - 1.0) * z * p1 - (k - 1.0) * p0) / k;
        p0 = p1; p1 = p2;
      }
      if (n == 1) { p1 = z; p0 = 1.0; }
      pp = n * (z * p1 - p0) / (z * z - 1.0);
    }
    x[n - 1 - i] = 0.5 * (1.0 + z);
    w[n - 1 - i] = 1.0 / ((1.0 - z * z) * pp * pp);
  }
}

/* Default quadrature rule for polynomial degree m. Returns point count; pts [nq][tdim]. */
int ora_quadrature(int ct, int m, double* pts, double* wts) {
  int td = tdim_of(ct);
  if (m < 1) m = 1;
  if (!simplex(ct)) {
    int n = (m + 2) / 2;
    double x[32], w[32];
    gauss_legendre01(n, x, w);
    int q = 0;
    if (td == 2) {
      for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) {
          pts[2 * q] = x[i]; pts[2 * q + 1] = x[j]; wts[q] = w[i] * w[j]; ++q;
        }
    } else {
      for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j)
          for (int k = 0; k < n; ++k) {
            pts[3 * q] = x[i]; pts[3 * q + 1] = x[j]; pts[3 * q + 2] = x[k];
            wts[q] = w[i] * w[j] * w[k]; ++q;
          }
    }
    return q;
  }
  if (m == 1) {
    if (td == 2) { pts[0] = pts[1] = 1.0 / 3.0; wts[0] = 0.5; }
    else { pts[0] = pts[1] = pts[2] = 0.25; wts[0] = 1.0 / 6.0; }
    return 1;
  }
  if (m == 2) {
    if (td == 2) {
      const double a = 1.0 / 6.0, b = 2.0 / 3.0;
      double P[3][2] = {{a, a}, {a, b}, {b, a}};
      for (int q = 0; q < 3; ++q) { pts[2 * q] = P[q][0]; pts[2 * q + 1] = P[q][1]; wts[q] = 1.0 / 6.0; }
      return 3;
    } else {
      const double a = 0.1381966011250105, b = 0.5854101966249685;
      double P[4][3] = {{b, a, a}, {a, b, a}, {a, a, b}, {a, a, a}};
      for (int q = 0; q < 4; ++q) {
        for (int d = 0; d < 3; ++d) pts[3 * q + d] = P[q][d];
        wts[q] = 1.0 / 24.0;
      }
      return 4;
    }
  }
  /* higher degrees: collapsed (Duffy) Gauss-Legendre product rule, exact to degree m */
  {
    int n = (m + 2) / 2 + 1;
    double x[32], w[32];
    gauss_legendre01(n, x, w);
    int q = 0;
    if (td == 2) {
      for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) {
          double u = x[i], v = x[j];
          pts[2 * q] = u * (1.0 - v); pts[2 * q + 1] = v;
          wts[q] = w[i] * w[j] * (1.0 - v); ++q;
        }
    } else {
      for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j)
          for (int k = 0; k < n; ++k) {
            double u = x[i], v = x[j], t = x[k];
            pts[3 * q] = u * (1.0 - v) * (1.0 - t);
            pts[3 * q + 1] = v * (1.0 - t);
            pts[3 * q + 2] = t;
            wts[q] = w[i] * w[j] * w[k] * (1.0 - v) * (1.0 - t) * (1.0 - t); ++q;
          }
    }
    return q;
  }
}

/* ---------------------------------------------------------------- geometry */
/* J[i][k] = sum_v x_v[i] dphi_v[k]; returns det J, fills Jinv (row-major [k][i]). */
static double jacobian(int gd, int nv, const double* gdphi /*[nv][gd]*/, const double* xv /*[nv][gd]*/,
                       double* Jinv) {
  double J[9] = {0};
  for (int v = 0; v < nv; ++v)
    for (int i = 0; i < gd; ++i)
      for (int k = 0; k < gd; ++k) J[i * 3 + k] += xv[v * gd + i] * gdphi[v * gd + k];
  double det;
  if (gd == 2) {
    det = J[0] * J[4] - J[1] * J[3];
    Jinv[0] = J[4] / det; Jinv[1] = -J[1] / det;
    Jinv[3] = -J[3] / det; Jinv[4] = J[0] / det;
  } else {
    det = J[0] * (J[4] * J[8] - J[5] * J[7]) - J[1] * (J[3] * J[8] - J[5] * J[6]) + J[2] * (J[3] * J[7] - J[4] * J[6]);
    Jinv[0] = (J[4] * J[8] - J[5] * J[7]) / det;
    Jinv[1] = (J[2] * J[7] - J[1] * J[8]) / det;
    Jinv[2] = (J[1] * J[5] - J[2] * J[4]) / det;
    Jinv[3] = (J[5] * J[6] - J[3] * J[8]) / det;
    Jinv[4] = (J[0] * J[8] - J[2] * J[6]) / det;
    Jinv[5] = (J[2] * J[3] - J[0] * J[5]) / det;
    Jinv[6] = (J[3] * J[7] - J[4] * J[6]) / det;
    Jinv[7] = (J[1] * J[6] - J[0] * J[7]) / det;
    Jinv[8] = (J[0] * J[4] - J[1] * J[3]) / det;
  }
  return det;
}

/* physical gradients g[n][d] = sum_k dphi[n][k] Jinv[k][d]  (MFEM: gdshape = dshape * InvJ) */
static void phys_grads(int gd, int nn, const double* dphi, const double* Jinv, double* g) {
  for (int n = 0; n < nn; ++n)
    for (int d = 0; d < gd; ++d) {
      double s = 0;
      for (int k = 0; k < gd; ++k) s += dphi[n * gd + k] * Jinv[k * 3 + d];
      g[n * gd + d] = s;
    }
}

/* Voigt strain-displacement matrix B [nvoigt][ndof], dof = node*gd + comp.
 * 2-D rows (xx, yy, xy); 3-D rows (xx, yy, zz, yz, xz, xy); engineering shear. */
static int voigt_B(int gd, int nn, const double* g, double* B) {
  int nv = gd == 2 ? 3 : 6, nd = nn * gd;
  memset(B, 0, sizeof(double) * nv * nd);
  for (int a = 0; a < nn; ++a) {
    const double* ga = &g[a * gd];
    if (gd == 2) {
      B[0 * nd + a * 2 + 0] = ga[0];
      B[1 * nd + a * 2 + 1] = ga[1];
      B[2 * nd + a * 2 + 0] = ga[1];
      B[2 * nd + a * 2 + 1] = ga[0];
    } else {
      B[0 * nd + a * 3 + 0] = ga[0];
      B[1 * nd + a * 3 + 1] = ga[1];
      B[2 * nd + a * 3 + 2] = ga[2];
      B[3 * nd + a * 3 + 1] = ga[2];
      B[3 * nd + a * 3 + 2] = ga[1];
      B[4 * nd + a * 3 + 0] = ga[2];
      B[4 * nd + a * 3 + 2] = ga[0];
      B[5 * nd + a * 3 + 0] = ga[1];
      B[5 * nd + a * 3 + 1] = ga[0];
    }
  }
  return nv;
}

static void hooke_D(int gd, double lam, double mu, double* D) {
  int nv = gd == 2 ? 3 : 6;
  memset(D, 0, sizeof(double) * nv * nv);
  for (int i = 0; i < gd; ++i) {
    for (int j = 0; j < gd; ++j) D[i * nv + j] = lam;
    D[i * nv + i] = lam + 2.0 * mu;
  }
  for (int i = gd; i < nv; ++i) D[i * nv + i] = mu;
}

/* Ae += sum_q w_q |det J_q| B_q^T D B_q   (dof = node*gd+comp). gdphi: geometry element
 * reference gradients at the same points [nq][nv][gd]. */
void ora_elasticity_cell(int gd, int nn, int nq, const double* wq, const double* dphi, int nv,
                         const double* gdphi, const double* xv, double lam, double mu, double* Ae) {
  int nd = nn * gd, nvo = gd == 2 ? 3 : 6;
  double Jinv[9], g[ORA_MAXN * 3], D[36];
  double* B = (double*)malloc(sizeof(double) * nvo * nd);
  double* DB = (double*)malloc(sizeof(double) * nvo * nd);
  hooke_D(gd, lam, mu, D);
  for (int q = 0; q < nq; ++q) {
    double det = jacobian(gd, nv, &gdphi[q * nv * gd], xv, Jinv);
    double w = wq[q] * fabs(det);
    phys_grads(gd, nn, &dphi[q * nn * gd], Jinv, g);
    voigt_B(gd, nn, g, B);
    for (int k = 0; k < nvo; ++k)
      for (int j = 0; j < nd; ++j) {
        double s = 0;
        for (int l = 0; l < nvo; ++l) s += D[k * nvo + l] * B[l * nd + j];
        DB[k * nd + j] = s;
      }
    for (int i = 0; i < nd; ++i)
      for (int j = 0; j < nd; ++j) {
        double s = 0;
        for (int k = 0; k < nvo; ++k) s += B[k * nd + i] * DB[k * nd + j];
        Ae[i * nd + j] += w * s;
      }
  }
  free(B);
  free(DB);
}

/* ---------------------------------------------------------------- damage law (2-D) */
/* MFEM damIntegrator hand tangent, MFEM/mechanic2d/asym_elasto_damage_model.cc:735-881.
 * strain = (e11, e22, e12) tensor components; hook is 3x3 Voigt (xx, yy, xy-engineering). */
void ora_damage_hook(const double* strain, double l, double m, double d, double* hook) {
  const double limit = 1.e-12, mlimit = -1.e-12;
  double s00 = strain[0], s11 = strain[1], s01 = strain[2];
  memset(hook, 0, 9 * sizeof(double));
  if (d > 0.) {
    if (d > 1. - limit) d = 1. - limit; /* :739 */
    double I1 = s00 + s11;
    double I2 = s01 * s01 - s00 * s11;
    if (I1 > limit || I2 > limit || I1 < mlimit || I2 < mlimit) {
      double delta = I1 * I1 + 4 * I2;
      double r = sqrt(delta > 0. ? delta : 0.);
      double e1 = (I1 + r) / 2., e2 = (I1 - r) / 2.;
      double coss, sinn;
      if (r < limit) {
        double signe = (2 * s01 / (s00 - s11)) > 0. ? 1 : -1;
        coss = signe * sqrt(2.) / 2.;
        sinn = coss;
      } else {
        coss = (s00 - s11) / r;
        sinn = 2 * s01 / r;
      }
      double alpha1 = e1 >= 0 ? 1. : 0., alpha2 = e2 >= 0 ? 1. : 0., alpha = I1 >= 0 ? 1. : 0.;
      double factor = 2. * m, gamma = 0.5 * l / m;
      double c1 = 1. - alpha1 * d, c2 = 1. - alpha2 * d, c3 = 1. - alpha * d;
      double P[4] = {factor * (c1 + gamma * c3), factor * gamma * c3, factor * gamma * c3, factor * (c2 + gamma * c3)};
      double De[2][3] = {{0.5 * (1 + coss), 0.5 * (1 - coss), 0.5 * sinn},
                         {0.5 * (1 - coss), 0.5 * (1 + coss), -0.5 * sinn}};
      double cos2 = coss * coss, sin2 = sinn * sinn, sc = sinn * coss;
      double M[9] = {1. - cos2, -1. + cos2, -sc, -1. + cos2, 1. - cos2, sc, -sc, sc, 1 - sin2};
      for (int k = 0; k < 9; ++k) M[k] *= 0.5 * m;
      /* hook = dedeps^T P dedeps + q M */
      double q = (r >= limit) ? (I1 / r * (c1 - c2) + (c1 + c2)) : (c1 + c2);
      for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
          double s = 0;
          for (int a = 0; a < 2; ++a)
            for (int b = 0; b < 2; ++b) s += De[a][i] * P[a * 2 + b] * De[b][j];
          hook[i * 3 + j] = s + q * M[i * 3 + j];
        }
    } else {
      double md = (1. - d) * m, ld = (1. - d) * l;
      hook[0] = hook[4] = 2 * md + ld;
      hook[1] = hook[3] = ld;
      hook[8] = md;
    }
  } else {
    hook[0] = hook[4] = 2 * m + l;
    hook[1] = hook[3] = l;
    hook[8] = m;
  }
}

/* asym_stress, hand version, MFEM/mechanic2d/asym_elasto_damage_model.cc:207-329.
 * Returns sig = (s00, s11, s01) already multiplied by w. */
void ora_damage_stress(const double* strain, double l, double m, double d, double w, double* sig) {
  const double limit = 1.e-12, mlimit = -1.e-12;
  double s00 = strain[0], s11 = strain[1], s01 = strain[2];
  if (d > 0.) {
    double I1 = s00 + s11, I2 = s01 * s01 - s00 * s11;
    if (I1 > limit || I2 > limit || I1 < mlimit || I2 < mlimit) {
      double delta = I1 * I1 + 4 * I2;
      double r = sqrt(delta > 0. ? delta : 0.);
      double ev[2] = {(I1 + r) / 2., (I1 - r) / 2.};
      double alpha1 = ev[0] >= 0 ? 1. : 0., alpha2 = ev[1] >= 0 ? 1. : 0.;
      double alpha = (ev[0] + ev[1]) >= 0 ? 1. : 0.;
      if (!((d == 1.) && (alpha == 1) && (alpha1 == 1) && (alpha2 == 1))) {
        double V[2][2];
        if (fabs(s01) > limit) {
          V[0][0] = ev[0] - s11; V[0][1] = ev[1] - s11;
          V[1][0] = V[1][1] = s01;
          double n0 = sqrt(V[0][0] * V[0][0] + V[1][0] * V[1][0]);
          double n1 = sqrt(V[0][1] * V[0][1] + V[1][1] * V[1][1]);
          V[0][0] /= n0; V[1][0] /= n0; V[0][1] /= n1; V[1][1] /= n1;
        } else {
          V[0][0] = V[1][1] = 1.; V[1][0] = V[0][1] = 0.;
        }
        double temp = 2. * m * w, gamma = 0.5 * l / m;
        double c = 1 - alpha * d, c1 = 1 - alpha1 * d, c2 = 1 - alpha2 * d;
        double D0 = temp * (c1 + gamma * c), D1 = temp * gamma * c, D2 = temp * (c2 + gamma * c);
        double es[2] = {D0 * ev[0] + D1 * ev[1], D1 * ev[0] + D2 * ev[1]};
        /* sig = V diag(es) V^T */
        sig[0] = V[0][0] * es[0] * V[0][0] + V[0][1] * es[1] * V[0][1];
        sig[1] = V[1][0] * es[0] * V[1][0] + V[1][1] * es[1] * V[1][1];
        sig[2] = V[0][0] * es[0] * V[1][0] + V[0][1] * es[1] * V[1][1];
      } else {
        sig[0] = sig[1] = sig[2] = 0.;
      }
    } else {
      sig[0] = sig[1] = sig[2] = 0.;
    }
  } else {
    double m2plw = w * (2 * m + l), lw = l * w;
    sig[0] = m2plw * s00 + lw * s11;
    sig[1] = m2plw * s11 + lw * s00;
    sig[2] = w * m * (s01 + s01);
  }
}

/* Damage-law P1 triangle tangent (one quadrature point, the centroid — `dxx` degree 1,
 * FEniCSx/mechanic2d/asym_ufl.py:78). d_cell = damage at the quadrature point, u_cell = the
 * element displacement, dolfinx-blocked [node][comp]. Ae += w * B hook B^T. */
void ora_damage_cell(const double* xv /*[3][2]*/, const double* u_cell /*[6]*/, double d_cell, double l, double m,
                     double* Ae) {
  const double dphi[3][2] = {{-1, -1}, {1, 0}, {0, 1}};
  double Jinv[9], g[6], B[3 * 6], hook[9];
  double det = jacobian(2, 3, &dphi[0][0], xv, Jinv);
  double w = 0.5 * fabs(det);
  phys_grads(2, 3, &dphi[0][0], Jinv, g);
  double grad[2][2] = {{0, 0}, {0, 0}}; /* grad[i][j] = du_i/dx_j */
  for (int a = 0; a < 3; ++a)
    for (int i = 0; i < 2; ++i)
      for (int j = 0; j < 2; ++j) grad[i][j] += u_cell[a * 2 + i] * g[a * 2 + j];
  double strain[3] = {grad[0][0], grad[1][1], 0.5 * (grad[0][1] + grad[1][0])};
  ora_damage_hook(strain, l, m, d_cell, hook);
  voigt_B(2, 3, g, B);
  for (int i = 0; i < 6; ++i)
    for (int j = 0; j < 6; ++j) {
      double s = 0;
      for (int k = 0; k < 3; ++k)
        for (int kk = 0; kk < 3; ++kk) s += B[k * 6 + i] * hook[k * 3 + kk] * B[kk * 6 + j];
      Ae[i * 6 + j] += w * s;
    }
}

/* ---------------------------------------------------------------- global assembly */
static int64_t find_col(const int64_t* indptr, const int32_t* indices, int64_t row, int32_t col) {
  int64_t lo = indptr[row], hi = indptr[row + 1] - 1;
  while (lo <= hi) {
    int64_t mid = (lo + hi) >> 1;
    int32_t c = indices[mid];
    if (c == col) return mid;
    if (c < col) lo = mid + 1; else hi = mid - 1;
  }
  return -1;
}

/* Sparsity (block/node level): all node pairs of every cell, sorted and unique per row.
 * Two-pass: call with indices == NULL to get indptr (size nnodes+1); then again to fill.
 * Returns the number of blocks, or -1 on failure. */
static int cmp_i64(const void* a, const void* b) {
  int64_t x = *(const int64_t*)a, y = *(const int64_t*)b;
  return (x > y) - (x < y);
}
int64_t ora_sparsity(int64_t nc, int nn, const int32_t* cells, int64_t nnodes, int64_t* indptr, int32_t* indices) {
  int64_t np = nc * nn * nn;
  int64_t* keys = (int64_t*)malloc(sizeof(int64_t) * (np > 0 ? np : 1));
  if (!keys) return -1;
  int64_t k = 0;
  for (int64_t c = 0; c < nc; ++c)
    for (int a = 0; a < nn; ++a)
      for (int b = 0; b < nn; ++b) keys[k++] = (int64_t)cells[c * nn + a] * nnodes + cells[c * nn + b];
  qsort(keys, (size_t)np, sizeof(int64_t), cmp_i64);
  int64_t u = 0;
  for (int64_t i = 0; i < np; ++i)
    if (i == 0 || keys[i] != keys[i - 1]) keys[u++] = keys[i];
  for (int64_t r = 0; r <= nnodes; ++r) indptr[r] = 0;
  for (int64_t i = 0; i < u; ++i) indptr[keys[i] / nnodes + 1]++;
  for (int64_t r = 0; r < nnodes; ++r) indptr[r + 1] += indptr[r];
  if (indices)
    for (int64_t i = 0; i < u; ++i) indices[i] = (int32_t)(keys[i] % nnodes);
  free(keys);
  return u;
}

typedef struct {
  int cell_type;
  int degree;      /* function-space degree */
  int gdim;        /* = tdim; also the block size bs */
  int64_t ncells;
  int nn;          /* nodes per cell */
  const int32_t* cells; /* [nc][nn] dofmap (node level) */
  int nv;          /* geometry nodes per cell (P1/Q1 vertices) */
  const int32_t* geom;  /* [nc][nv] */
  const double* x;      /* [nverts][gdim] */
} ora_mesh;

/* Linear-elasticity matrix assembly into a BSR matrix (block = gdim x gdim, row-major).
 * lam/mu per cell. bc: int8 per dof (node*bs+comp) or NULL. qdeg < 0 -> estimated degree
 * (2*(p-1) on simplices, 2*p on tensor cells, as UFL estimates it for this form).
 * dolfinx semantics: values are ADDED (caller zeroes), bc rows/cols zeroed in A_e, then
 * `diag` INSERTED on bc diagonal entries (set_diagonal). Returns 0 or a negative error. */
int ora_assemble_elasticity(const ora_mesh* M, const double* lam, const double* mu, int qdeg, const int8_t* bc,
                            double diag, const int64_t* indptr, const int32_t* indices, double* values) {
  int gd = M->gdim, nn = M->nn, nv = M->nv, bs = gd;
  int tdim = gd;
  if (qdeg < 0) qdeg = simplex(M->cell_type) ? 2 * (M->degree - 1) : 2 * M->degree;
  static double pts[ORA_MAXQ * 3], wq[ORA_MAXQ];
  int nq = ora_quadrature(M->cell_type, qdeg, pts, wq);
  double* dphi = (double*)malloc(sizeof(double) * nq * nn * tdim);
  double* gdphi = (double*)malloc(sizeof(double) * nq * nv * tdim);
  if (ora_tabulate(M->cell_type, M->degree, nq, pts, NULL, dphi) != nn) return -2;
  if (ora_tabulate(M->cell_type, 1, nq, pts, NULL, gdphi) != nv) return -3;
  int nd = nn * bs;
  double* Ae = (double*)malloc(sizeof(double) * nd * nd);
  double xv[8 * 3];
  for (int64_t c = 0; c < M->ncells; ++c) {
    memset(Ae, 0, sizeof(double) * nd * nd);
    for (int v = 0; v < nv; ++v)
      for (int d = 0; d < gd; ++d) xv[v * gd + d] = M->x[(int64_t)M->geom[c * nv + v] * gd + d];
    ora_elasticity_cell(gd, nn, nq, wq, dphi, nv, gdphi, xv, lam[c], mu[c], Ae);
    const int32_t* nodes = &M->cells[c * nn];
    if (bc)
      for (int i = 0; i < nd; ++i)
        if (bc[(int64_t)nodes[i / bs] * bs + i % bs])
          for (int j = 0; j < nd; ++j) Ae[i * nd + j] = Ae[j * nd + i] = 0.0;
    for (int a = 0; a < nn; ++a)
      for (int b = 0; b < nn; ++b) {
        int64_t s = find_col(indptr, indices, nodes[a], nodes[b]);
        if (s < 0) { free(Ae); free(dphi); free(gdphi); return -4; }
        double* blk = &values[s * bs * bs];
        for (int i = 0; i < bs; ++i)
          for (int j = 0; j < bs; ++j) blk[i * bs + j] += Ae[(a * bs + i) * nd + b * bs + j];
      }
  }
  free(Ae); free(dphi); free(gdphi);
  if (bc) {
    int64_t nnodes = 0;
    for (int64_t c = 0; c < M->ncells * nn; ++c)
      if (M->cells[c] + 1 > nnodes) nnodes = M->cells[c] + 1;
    for (int64_t r = 0; r < nnodes; ++r)
      for (int i = 0; i < bs; ++i)
        if (bc[r * bs + i]) {
          int64_t s = find_col(indptr, indices, r, (int32_t)r);
          if (s >= 0) values[s * bs * bs + i * bs + i] = diag;
        }
  }
  return 0;
}

/* Damage-law Jacobian assembly (P1 triangles, 2-D): the reference mechanic2d J form.
 * u: displacement per dof (node*2+comp); dnode: damage per vertex (P1). lam/mu per cell. */
int ora_assemble_damage(const ora_mesh* M, const double* lam, const double* mu, const double* u, const double* dnode,
                        const int8_t* bc, double diag, const int64_t* indptr, const int32_t* indices, double* values) {
  if (M->cell_type != ORA_TRI || M->degree != 1) return -1;
  double Ae[36], xv[6], uc[6];
  for (int64_t c = 0; c < M->ncells; ++c) {
    const int32_t* nodes = &M->cells[c * 3];
    memset(Ae, 0, sizeof Ae);
    double dq = 0;
    for (int v = 0; v < 3; ++v) {
      for (int d = 0; d < 2; ++d) {
        xv[v * 2 + d] = M->x[(int64_t)M->geom[c * 3 + v] * 2 + d];
        uc[v * 2 + d] = u[(int64_t)nodes[v] * 2 + d];
      }
      dq += dnode[nodes[v]] / 3.0;
    }
    ora_damage_cell(xv, uc, dq, lam[c], mu[c], Ae);
    if (bc)
      for (int i = 0; i < 6; ++i)
        if (bc[(int64_t)nodes[i / 2] * 2 + i % 2])
          for (int j = 0; j < 6; ++j) Ae[i * 6 + j] = Ae[j * 6 + i] = 0.0;
    for (int a = 0; a < 3; ++a)
      for (int b = 0; b < 3; ++b) {
        int64_t s = find_col(indptr, indices, nodes[a], nodes[b]);
        if (s < 0) return -4;
        for (int i = 0; i < 2; ++i)
          for (int j = 0; j < 2; ++j) values[s * 4 + i * 2 + j] += Ae[(a * 2 + i) * 6 + b * 2 + j];
      }
  }
  if (bc) {
    int64_t nnodes = 0;
    for (int64_t c = 0; c < M->ncells * 3; ++c)
      if (M->cells[c] + 1 > nnodes) nnodes = M->cells[c] + 1;
    for (int64_t r = 0; r < nnodes; ++r)
      for (int i = 0; i < 2; ++i)
        if (bc[r * 2 + i]) {
          int64_t s = find_col(indptr, indices, r, (int32_t)r);
          if (s >= 0) values[s * 4 + i * 2 + i] = diag;
        }
  }
  return 0;
}

/* Element matrices only (the ffcx tabulate_tensor / MFEM AssembleElementGrad level):
 * Ae[nc][nd][nd], no bc. Used to check the device per-cell kernel directly. */
int ora_cell_matrices_elasticity(const ora_mesh* M, const double* lam, const double* mu, int qdeg, double* Aout) {
  int gd = M->gdim, nn = M->nn, nv = M->nv, nd = nn * gd;
  if (qdeg < 0) qdeg = simplex(M->cell_type) ? 2 * (M->degree - 1) : 2 * M->degree;
  static double pts[ORA_MAXQ * 3], wq[ORA_MAXQ];
  int nq = ora_quadrature(M->cell_type, qdeg, pts, wq);
  double* dphi = (double*)malloc(sizeof(double) * nq * nn * gd);
  double* gdphi = (double*)malloc(sizeof(double) * nq * nv * gd);
  if (ora_tabulate(M->cell_type, M->degree, nq, pts, NULL, dphi) != nn) return -2;
  if (ora_tabulate(M->cell_type, 1, nq, pts, NULL, gdphi) != nv) return -3;
  double xv[8 * 3];
  for (int64_t c = 0; c < M->ncells; ++c) {
    double* Ae = &Aout[c * nd * nd];
    memset(Ae, 0, sizeof(double) * nd * nd);
    for (int v = 0; v < nv; ++v)
      for (int d = 0; d < gd; ++d) xv[v * gd + d] = M->x[(int64_t)M->geom[c * nv + v] * gd + d];
    ora_elasticity_cell(gd, nn, nq, wq, dphi, nv, gdphi, xv, lam[c], mu[c], Ae);
  }
  free(dphi); free(gdphi);
  return 0;
}

/* ---------------------------------------------------------------- residual & lifting */
static void neo_stress(int gd, const double* F, double lam, double mu, double* P);
static void neo_cell(int gd, int nn, int nq, const double* wq, const double* dphi, int nv, const double* gdphi,
                     const double* xv, const double* uc, double lam, double mu, double* Ae);
/* dolfinx assemble_vector of F = inner(sigma(u), eps(v)) dx_qs - inner(f, v) dx_qf restated
 * per cell with Voigt vectors: b_e = sum_q w|J| B^T sigma_v - sum_q w|J| N^T f(q); b[dofs] += b_e.
 * kind 0: linear sigma = D B u;  kind 1: reference damage law (P1 tri, centroid, asym_stress);
 * kind 2: neo-Hookean, b_e[a,i] = sum_q w|J| P_iJ(F_q) g_a[J] with F_q = I + grad u.
 * u, f per dof (may be NULL); dnode per node (kind 1). qs < 0: estimated degree. */
int ora_assemble_residual(const ora_mesh* M, int kind, const double* lam, const double* mu, const double* u,
                          const double* dnode, const double* f, int qs, double* b) {
  int gd = M->gdim, nn = M->nn, nv = M->nv, nd = nn * gd, nvo = gd == 2 ? 3 : 6;
  if (qs < 0) qs = simplex(M->cell_type) ? 2 * (M->degree - 1) : 2 * M->degree;
  if (kind == 1) qs = 1;
  int qf = 2 * M->degree;
  static double ps[ORA_MAXQ * 3], ws[ORA_MAXQ], pf[ORA_MAXQ * 3], wf[ORA_MAXQ];
  int nqs = ora_quadrature(M->cell_type, qs, ps, ws);
  int nqf = ora_quadrature(M->cell_type, qf, pf, wf);
  double* dphi_s = (double*)malloc(sizeof(double) * nqs * nn * gd);
  double* gdphi_s = (double*)malloc(sizeof(double) * nqs * nv * gd);
  double* phi_f = (double*)malloc(sizeof(double) * nqf * nn);
  double* gdphi_f = (double*)malloc(sizeof(double) * nqf * nv * gd);
  ora_tabulate(M->cell_type, M->degree, nqs, ps, NULL, dphi_s);
  ora_tabulate(M->cell_type, 1, nqs, ps, NULL, gdphi_s);
  ora_tabulate(M->cell_type, M->degree, nqf, pf, phi_f, NULL);
  ora_tabulate(M->cell_type, 1, nqf, pf, NULL, gdphi_f);
  double* be = (double*)malloc(sizeof(double) * nd);
  double* B = (double*)malloc(sizeof(double) * nvo * nd);
  double Jinv[9], g[ORA_MAXN * 3], D[36], xv[8 * 3];
  for (int64_t c = 0; c < M->ncells; ++c) {
    const int32_t* nodes = &M->cells[c * nn];
    memset(be, 0, sizeof(double) * nd);
    for (int v = 0; v < nv; ++v)
      for (int d = 0; d < gd; ++d) xv[v * gd + d] = M->x[(int64_t)M->geom[c * nv + v] * gd + d];
    if (u) {
      for (int q = 0; q < nqs; ++q) {
        double det = jacobian(gd, nv, &gdphi_s[q * nv * gd], xv, Jinv);
        double w = ws[q] * fabs(det);
        phys_grads(gd, nn, &dphi_s[q * nn * gd], Jinv, g);
        voigt_B(gd, nn, g, B);
        double ev[6] = {0}, sv[6] = {0};
        for (int k = 0; k < nvo; ++k)
          for (int j = 0; j < nd; ++j) ev[k] += B[k * nd + j] * u[(int64_t)nodes[j / gd] * gd + j % gd];
        if (kind == 1) {
          double dq = 0;
          for (int a = 0; a < 3; ++a) dq += dnode[nodes[a]] / 3.0;
          double strain[3] = {ev[0], ev[1], 0.5 * ev[2]}, sig[3];
          ora_damage_stress(strain, lam[c], mu[c], dq, w, sig);
          sv[0] = sig[0]; sv[1] = sig[1]; sv[2] = sig[2];
          for (int i = 0; i < nd; ++i)
            for (int k = 0; k < nvo; ++k) be[i] += B[k * nd + i] * sv[k];
        } else if (kind == 2) {
          double F[9], P[9];
          for (int i = 0; i < gd; ++i)
            for (int k = 0; k < gd; ++k) {
              double s = (i == k) ? 1.0 : 0.0;
              for (int a = 0; a < nn; ++a) s += u[(int64_t)nodes[a] * gd + i] * g[a * gd + k];
              F[i * gd + k] = s;
            }
          neo_stress(gd, F, lam[c], mu[c], P);
          for (int a = 0; a < nn; ++a)
            for (int i = 0; i < gd; ++i)
              for (int k = 0; k < gd; ++k) be[a * gd + i] += w * P[i * gd + k] * g[a * gd + k];
        } else {
          hooke_D(gd, lam[c], mu[c], D);
          for (int k = 0; k < nvo; ++k)
            for (int l = 0; l < nvo; ++l) sv[k] += D[k * nvo + l] * ev[l];
          for (int i = 0; i < nd; ++i)
            for (int k = 0; k < nvo; ++k) be[i] += w * B[k * nd + i] * sv[k];
        }
      }
    }
    if (f) {
      for (int q = 0; q < nqf; ++q) {
        double det = jacobian(gd, nv, &gdphi_f[q * nv * gd], xv, Jinv);
        double w = wf[q] * fabs(det);
        double fq[3] = {0, 0, 0};
        for (int a = 0; a < nn; ++a)
          for (int i = 0; i < gd; ++i) fq[i] += phi_f[q * nn + a] * f[(int64_t)nodes[a] * gd + i];
        for (int a = 0; a < nn; ++a)
          for (int i = 0; i < gd; ++i) be[a * gd + i] -= w * phi_f[q * nn + a] * fq[i];
      }
    }
    for (int i = 0; i < nd; ++i) b[(int64_t)nodes[i / gd] * gd + i % gd] += be[i];
  }
  free(be); free(B); free(dphi_s); free(gdphi_s); free(phi_f); free(gdphi_f);
  return 0;
}

/* dolfinx apply_lifting (one form, one bc set): for every cell holding a constrained dof,
 * b[dofs] -= alpha * A_e (g - x0) restricted to constrained columns (FEniCSx/mechanic2d/
 * asym_elasto_damage_model.cc:827 calls it with alpha = -1). kind as above (J form). */
int ora_apply_lifting(const ora_mesh* M, int kind, const double* lam, const double* mu, const double* u,
                      const double* dnode, int qdeg, const int8_t* bc, const double* gval, const double* x0,
                      double alpha, double* b) {
  int gd = M->gdim, nn = M->nn, nv = M->nv, nd = nn * gd;
  if (qdeg < 0) qdeg = simplex(M->cell_type) ? 2 * (M->degree - 1) : 2 * M->degree;
  static double pts[ORA_MAXQ * 3], wq[ORA_MAXQ];
  int nq = ora_quadrature(M->cell_type, qdeg, pts, wq);
  double* dphi = (double*)malloc(sizeof(double) * nq * nn * gd);
  double* gdphi = (double*)malloc(sizeof(double) * nq * nv * gd);
  ora_tabulate(M->cell_type, M->degree, nq, pts, NULL, dphi);
  ora_tabulate(M->cell_type, 1, nq, pts, NULL, gdphi);
  double* Ae = (double*)malloc(sizeof(double) * nd * nd);
  double xv[8 * 3], vbc[ORA_MAXN * 3];
  for (int64_t c = 0; c < M->ncells; ++c) {
    const int32_t* nodes = &M->cells[c * nn];
    int any = 0;
    for (int i = 0; i < nd; ++i) {
      int64_t dof = (int64_t)nodes[i / gd] * gd + i % gd;
      vbc[i] = bc[dof] ? gval[dof] - (x0 ? x0[dof] : 0.0) : 0.0;
      any |= bc[dof] != 0;
    }
    if (!any) continue;
    memset(Ae, 0, sizeof(double) * nd * nd);
    for (int v = 0; v < nv; ++v)
      for (int d = 0; d < gd; ++d) xv[v * gd + d] = M->x[(int64_t)M->geom[c * nv + v] * gd + d];
    if (kind == 1) {
      double uc[6], dq = 0;
      for (int a = 0; a < 3; ++a) {
        for (int d = 0; d < 2; ++d) uc[a * 2 + d] = u ? u[(int64_t)nodes[a] * 2 + d] : 0.0;
        dq += (dnode ? dnode[nodes[a]] : 0.0) / 3.0;
      }
      ora_damage_cell(xv, uc, dq, lam[c], mu[c], Ae);
    } else if (kind == 2) {
      double uc[ORA_MAXN * 3];
      for (int i = 0; i < nd; ++i) uc[i] = u[(int64_t)nodes[i / gd] * gd + i % gd];
      neo_cell(gd, nn, nq, wq, dphi, nv, gdphi, xv, uc, lam[c], mu[c], Ae);
    } else {
      ora_elasticity_cell(gd, nn, nq, wq, dphi, nv, gdphi, xv, lam[c], mu[c], Ae);
    }
    for (int i = 0; i < nd; ++i) {
      double s = 0;
      for (int j = 0; j < nd; ++j) s += Ae[i * nd + j] * vbc[j];
      b[(int64_t)nodes[i / gd] * gd + i % gd] -= alpha * s;
    }
  }
  free(Ae); free(dphi); free(gdphi);
  return 0;
}

/* ---------------------------------------------------------------- neo-Hookean (config E) */
/* psi(F) = mu/2 (I_C - 3) - mu ln J + lam/2 (ln J)^2 (2-D: plane strain). Closed-form tangent
 * (independent of the device's AD): with G = F^{-1},
 * A[(iJ)(kL)] = mu d_ik d_JL + (mu - lam ln J) G_Jk G_Li + lam G_Ji G_Lk. */
static double neo_inverse(int gd, const double* F, double* G) {
  double J;
  if (gd == 2) {
    J = F[0] * F[3] - F[1] * F[2];
    G[0] = F[3] / J; G[1] = -F[1] / J; G[2] = -F[2] / J; G[3] = F[0] / J;
  } else {
    J = F[0] * (F[4] * F[8] - F[5] * F[7]) - F[1] * (F[3] * F[8] - F[5] * F[6]) + F[2] * (F[3] * F[7] - F[4] * F[6]);
    G[0] = (F[4] * F[8] - F[5] * F[7]) / J;
    G[1] = (F[2] * F[7] - F[1] * F[8]) / J;
    G[2] = (F[1] * F[5] - F[2] * F[4]) / J;
    G[3] = (F[5] * F[6] - F[3] * F[8]) / J;
    G[4] = (F[0] * F[8] - F[2] * F[6]) / J;
    G[5] = (F[2] * F[3] - F[0] * F[5]) / J;
    G[6] = (F[3] * F[7] - F[4] * F[6]) / J;
    G[7] = (F[1] * F[6] - F[0] * F[7]) / J;
    G[8] = (F[0] * F[4] - F[1] * F[3]) / J;
  }
  return J;
}

/* First Piola stress P = d psi / dF = mu (F - F^{-T}) + lam ln J F^{-T}. */
static void neo_stress(int gd, const double* F, double lam, double mu, double* P) {
  double G[9];
  double lnJ = log(neo_inverse(gd, F, G));
  for (int i = 0; i < gd; ++i)
    for (int Jx = 0; Jx < gd; ++Jx) P[i * gd + Jx] = mu * F[i * gd + Jx] + (lam * lnJ - mu) * G[Jx * gd + i];
}

static void neo_tangent(int gd, const double* F, double lam, double mu, double* A) {
  double G[9];
  double J = neo_inverse(gd, F, G);
  double lnJ = log(J);
  int N = gd * gd;
  for (int i = 0; i < gd; ++i)
    for (int Jx = 0; Jx < gd; ++Jx)
      for (int k = 0; k < gd; ++k)
        for (int L = 0; L < gd; ++L)
          A[(i * gd + Jx) * N + k * gd + L] = ((i == k && Jx == L) ? mu : 0.0) +
                                              (mu - lam * lnJ) * G[Jx * gd + k] * G[L * gd + i] +
                                              lam * G[Jx * gd + i] * G[L * gd + k];
}

/* K[(a,i),(b,k)] += sum_q w|J| sum_{J,L} g_a[J] A_q[(iJ)(kL)] g_b[L], F_q = I + sum_b u_b (x) g_b(q) */
static void neo_cell(int gd, int nn, int nq, const double* wq, const double* dphi, int nv, const double* gdphi,
                     const double* xv, const double* uc, double lam, double mu, double* Ae) {
  int nd = nn * gd, N = gd * gd;
  double Jinv[9], g[ORA_MAXN * 3], F[9], A[81];
  for (int q = 0; q < nq; ++q) {
    double det = jacobian(gd, nv, &gdphi[q * nv * gd], xv, Jinv);
    double w = wq[q] * fabs(det);
    phys_grads(gd, nn, &dphi[q * nn * gd], Jinv, g);
    for (int i = 0; i < gd; ++i)
      for (int k = 0; k < gd; ++k) {
        double s = (i == k) ? 1.0 : 0.0;
        for (int b = 0; b < nn; ++b) s += uc[b * gd + i] * g[b * gd + k];
        F[i * gd + k] = s;
      }
    neo_tangent(gd, F, lam, mu, A);
    for (int a = 0; a < nn; ++a)
      for (int b = 0; b < nn; ++b)
        for (int i = 0; i < gd; ++i)
          for (int k = 0; k < gd; ++k) {
            double s = 0;
            for (int Jx = 0; Jx < gd; ++Jx)
              for (int L = 0; L < gd; ++L) s += g[a * gd + Jx] * A[(i * gd + Jx) * N + k * gd + L] * g[b * gd + L];
            Ae[(a * gd + i) * nd + b * gd + k] += w * s;
          }
  }
}

/* neo-Hookean tangent assembly (dolfinx semantics, as ora_assemble_elasticity); also returns the
 * cell matrices when Aout != NULL (then indptr/indices/values may be NULL). */
int ora_assemble_neohookean(const ora_mesh* M, const double* lam, const double* mu, const double* u, int qdeg,
                            const int8_t* bc, double diag, const int64_t* indptr, const int32_t* indices,
                            double* values, double* Aout) {
  int gd = M->gdim, nn = M->nn, nv = M->nv, bs = gd, nd = nn * gd;
  if (qdeg < 0) qdeg = simplex(M->cell_type) ? 2 * (M->degree - 1) : 2 * M->degree;
  static double pts[ORA_MAXQ * 3], wq[ORA_MAXQ];
  int nq = ora_quadrature(M->cell_type, qdeg, pts, wq);
  double* dphi = (double*)malloc(sizeof(double) * nq * nn * gd);
  double* gdphi = (double*)malloc(sizeof(double) * nq * nv * gd);
  ora_tabulate(M->cell_type, M->degree, nq, pts, NULL, dphi);
  ora_tabulate(M->cell_type, 1, nq, pts, NULL, gdphi);
  double* Ae = (double*)malloc(sizeof(double) * nd * nd);
  double xv[8 * 3], uc[ORA_MAXN * 3];
  for (int64_t c = 0; c < M->ncells; ++c) {
    const int32_t* nodes = &M->cells[c * nn];
    memset(Ae, 0, sizeof(double) * nd * nd);
    for (int v = 0; v < nv; ++v)
      for (int d = 0; d < gd; ++d) xv[v * gd + d] = M->x[(int64_t)M->geom[c * nv + v] * gd + d];
    for (int a = 0; a < nn; ++a)
      for (int d = 0; d < gd; ++d) uc[a * gd + d] = u[(int64_t)nodes[a] * gd + d];
    neo_cell(gd, nn, nq, wq, dphi, nv, gdphi, xv, uc, lam[c], mu[c], Ae);
    if (Aout) {
      memcpy(&Aout[c * nd * nd], Ae, sizeof(double) * nd * nd);
      continue;
    }
    if (bc)
      for (int i = 0; i < nd; ++i)
        if (bc[(int64_t)nodes[i / bs] * bs + i % bs])
          for (int j = 0; j < nd; ++j) Ae[i * nd + j] = Ae[j * nd + i] = 0.0;
    for (int a = 0; a < nn; ++a)
      for (int b = 0; b < nn; ++b) {
        int64_t s = find_col(indptr, indices, nodes[a], nodes[b]);
        if (s < 0) { free(Ae); free(dphi); free(gdphi); return -4; }
        for (int i = 0; i < bs; ++i)
          for (int j = 0; j < bs; ++j) values[s * bs * bs + i * bs + j] += Ae[(a * bs + i) * nd + b * bs + j];
      }
  }
  free(Ae); free(dphi); free(gdphi);
  if (bc && !Aout) {
    int64_t nnodes = 0;
    for (int64_t c = 0; c < M->ncells * nn; ++c)
      if (M->cells[c] + 1 > nnodes) nnodes = M->cells[c] + 1;
    for (int64_t r = 0; r < nnodes; ++r)
      for (int i = 0; i < bs; ++i)
        if (bc[r * bs + i]) {
          int64_t s = find_col(indptr, indices, r, (int32_t)r);
          if (s >= 0) values[s * bs * bs + i * bs + i] = diag;
        }
  }
  return 0;
}

/* public wrapper for tests */
void ora_neo_tangent(int gd, const double* F, double lam, double mu, double* A) { neo_tangent(gd, F, lam, mu, A); }
void ora_neo_stress(int gd, const double* F, double lam, double mu, double* P) { neo_stress(gd, F, lam, mu, P); }

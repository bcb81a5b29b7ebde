// Host-side element definitions for femasm: Lagrange basis tables and quadrature rules.
//
// Restates basix 0.8 (3rd-party, the element library behind the reference's UFL forms,
// FEniCSx/mechanic2d/asym_ufl.py:11-13 and doc.tex:511-536) for the cells the hot path
// supports, with basix's local node ordering (vertices, then edge, face and cell
// interiors; edges and faces in basix reference-cell order):
//   simplex P1/P2  closed-form barycentric basis;
//   tensor Q1..Q3  products of 1-D Lagrange polynomials on equispaced points (p <= 2) or
//                  GLL points (p = 3, basix's default gll_warped variant).
// Quadrature mirrors basix's default rule: Xiao-Gimbutas for simplex degree <= 2 (the
// degrees the reference's forms use), a collapsed Gauss-Legendre product above that, and
// Gauss-Legendre with (m+2)/2 points per direction on quadrilaterals/hexahedra.
// The tables are computed once per (cell, degree, quadrature degree) and copied to the
// device; kernels stage them in LDS.
#pragma once
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

namespace femasm {

enum CellType : int32_t { kTriangle = 3, kQuadrilateral = 4, kTetrahedron = -4, kHexahedron = 8 };

inline bool is_simplex(int ct) { return ct == kTriangle || ct == kTetrahedron; }
inline int cell_tdim(int ct) { return (ct == kTriangle || ct == kQuadrilateral) ? 2 : 3; }
inline int cell_nverts(int ct) {
  switch (ct) {
    case kTriangle: return 3;
    case kQuadrilateral: return 4;
    case kTetrahedron: return 4;
    case kHexahedron: return 8;
  }
  return 0;
}
inline int num_nodes(int ct, int p) {
  switch (ct) {
    case kTriangle: return (p + 1) * (p + 2) / 2;
    case kTetrahedron: return (p + 1) * (p + 2) * (p + 3) / 6;
    case kQuadrilateral: return (p + 1) * (p + 1);
    case kHexahedron: return (p + 1) * (p + 1) * (p + 1);
  }
  return 0;
}
inline bool supported(int ct, int p) {
  if (is_simplex(ct)) return p == 1 || p == 2;
  if (ct == kQuadrilateral || ct == kHexahedron) return p >= 1 && p <= 3;
  return false;
}

// Quadrature degree UFL estimates for the linear-elasticity bilinear form
// inner(sigma(du), eps(v)) on affine simplices (gradients drop one degree) and on
// tensor cells (UFL does not drop the degree of a tensor-product element's gradient).
inline int estimated_qdeg(int ct, int p) { return is_simplex(ct) ? 2 * (p - 1) : 2 * p; }

struct Quadrature {
  int tdim = 0;
  std::vector<double> pts;  // [nq][tdim]
  std::vector<double> wts;  // [nq]
  int size() const { return (int)wts.size(); }
};

inline void gauss_legendre_01(int n, std::vector<double>& x, std::vector<double>& w) {
  // Golub-Welsch would need an eigensolver; Newton on the Legendre recurrence is exact to
  // machine precision for the n <= 16 used here.
  x.assign(n, 0.0);
  w.assign(n, 0.0);
  for (int i = 0; i < n; ++i) {
    double z = std::cos(M_PI * (i + 0.75) / (n + 0.5));
    double dp = 1.0;
    for (int it = 0; it < 64; ++it) {
      double p0 = 1.0, p1 = z;
      for (int k = 2; k <= n; ++k) {
        double p2 = ((2.0 * k - 1.0) * z * p1 - (k - 1.0) * p0) / k;
        p0 = p1;
        p1 = p2;
      }
      if (n == 1) { p0 = 1.0; p1 = z; }
      dp = n * (z * p1 - p0) / (z * z - 1.0);
      double step = p1 / dp;
      z -= step;
      if (std::fabs(step) < 1e-17) break;
    }
    double p0 = 1.0, p1 = z;
    for (int k = 2; k <= n; ++k) {
      double p2 = ((2.0 * k - 1.0) * z * p1 - (k - 1.0) * p0) / k;
      p0 = p1;
      p1 = p2;
    }
    if (n == 1) { p0 = 1.0; p1 = z; }
    dp = n * (z * p1 - p0) / (z * z - 1.0);
    // ascending order on [0,1]
    x[n - 1 - i] = 0.5 * (1.0 + z);
    w[n - 1 - i] = 1.0 / ((1.0 - z * z) * dp * dp);
  }
}

inline Quadrature make_quadrature(int ct, int m) {
  Quadrature Q;
  Q.tdim = cell_tdim(ct);
  if (m < 1) m = 1;
  if (!is_simplex(ct)) {
    std::vector<double> x, w;
    gauss_legendre_01((m + 2) / 2, x, w);
    int n = (int)x.size();
    if (Q.tdim == 2) {
      for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) {
          Q.pts.push_back(x[i]);
          Q.pts.push_back(x[j]);
          Q.wts.push_back(w[i] * w[j]);
        }
    } else {
      for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j)
          for (int k = 0; k < n; ++k) {
            Q.pts.push_back(x[i]);
            Q.pts.push_back(x[j]);
            Q.pts.push_back(x[k]);
            Q.wts.push_back(w[i] * w[j] * w[k]);
          }
    }
    return Q;
  }
  if (m == 1) {
    if (Q.tdim == 2) Q.pts = {1.0 / 3.0, 1.0 / 3.0}, Q.wts = {0.5};
    else Q.pts = {0.25, 0.25, 0.25}, Q.wts = {1.0 / 6.0};
    return Q;
  }
  if (m == 2) {  // Xiao-Gimbutas degree 2
    if (Q.tdim == 2) {
      const double a = 1.0 / 6.0, b = 2.0 / 3.0;
      Q.pts = {a, a, a, b, b, a};
      Q.wts = {1.0 / 6.0, 1.0 / 6.0, 1.0 / 6.0};
    } else {
      const double a = 0.1381966011250105, b = 0.5854101966249685;
      Q.pts = {b, a, a, a, b, a, a, a, b, a, a, a};
      Q.wts = {1.0 / 24.0, 1.0 / 24.0, 1.0 / 24.0, 1.0 / 24.0};
    }
    return Q;
  }
  // collapsed (Duffy) Gauss-Legendre product, exact to degree m
  std::vector<double> x, w;
  gauss_legendre_01((m + 2) / 2 + 1, x, w);
  int n = (int)x.size();
  if (Q.tdim == 2) {
    for (int i = 0; i < n; ++i)
      for (int j = 0; j < n; ++j) {
        Q.pts.push_back(x[i] * (1.0 - x[j]));
        Q.pts.push_back(x[j]);
        Q.wts.push_back(w[i] * w[j] * (1.0 - x[j]));
      }
  } else {
    for (int i = 0; i < n; ++i)
      for (int j = 0; j < n; ++j)
        for (int k = 0; k < n; ++k) {
          double u = x[i], v = x[j], t = x[k];
          Q.pts.push_back(u * (1.0 - v) * (1.0 - t));
          Q.pts.push_back(v * (1.0 - t));
          Q.pts.push_back(t);
          Q.wts.push_back(w[i] * w[j] * w[k] * (1.0 - v) * (1.0 - t) * (1.0 - t));
        }
  }
  return Q;
}

// 1-D node set of a tensor element of degree p, in lattice order 0..p.
inline std::vector<double> line_points(int p) {
  if (p == 3) return {0.0, 0.5 * (1.0 - 1.0 / std::sqrt(5.0)), 0.5 * (1.0 + 1.0 / std::sqrt(5.0)), 1.0};
  std::vector<double> r(p + 1);
  for (int i = 0; i <= p; ++i) r[i] = (double)i / p;
  return r;
}

// basix local node -> lattice index (i, j, k) in 0..p for quadrilaterals / hexahedra.
inline std::vector<int> tensor_node_lattice(int ct, int p) {
  std::vector<int> L;  // [nn][3]
  auto push = [&](int i, int j, int k) { L.push_back(i); L.push_back(j); L.push_back(k); };
  if (ct == kQuadrilateral) {
    const int V[4][2] = {{0, 0}, {1, 0}, {0, 1}, {1, 1}};
    const int E[4][2] = {{0, 1}, {0, 2}, {1, 3}, {2, 3}};
    for (auto& v : V) push(v[0] * p, v[1] * p, 0);
    for (auto& e : E)
      for (int s = 1; s < p; ++s)
        push(V[e[0]][0] * p + s * (V[e[1]][0] - V[e[0]][0]), V[e[0]][1] * p + s * (V[e[1]][1] - V[e[0]][1]), 0);
    for (int i = 1; i < p; ++i)
      for (int j = 1; j < p; ++j) push(i, j, 0);
    return L;
  }
  const int V[8][3] = {{0, 0, 0}, {1, 0, 0}, {0, 1, 0}, {1, 1, 0}, {0, 0, 1}, {1, 0, 1}, {0, 1, 1}, {1, 1, 1}};
  const int E[12][2] = {{0, 1}, {0, 2}, {0, 4}, {1, 3}, {1, 5}, {2, 3}, {2, 6}, {3, 7}, {4, 5}, {4, 6}, {5, 7}, {6, 7}};
  const int F[6][3] = {{0, 1, 2}, {0, 1, 4}, {0, 2, 4}, {1, 3, 5}, {2, 3, 6}, {4, 5, 6}};
  for (auto& v : V) push(v[0] * p, v[1] * p, v[2] * p);
  for (auto& e : E)
    for (int s = 1; s < p; ++s) {
      int l[3];
      for (int d = 0; d < 3; ++d) l[d] = V[e[0]][d] * p + s * (V[e[1]][d] - V[e[0]][d]);
      push(l[0], l[1], l[2]);
    }
  for (auto& f : F)
    for (int s = 1; s < p; ++s)
      for (int t = 1; t < p; ++t) {
        int l[3];
        for (int d = 0; d < 3; ++d)
          l[d] = V[f[0]][d] * p + s * (V[f[1]][d] - V[f[0]][d]) + t * (V[f[2]][d] - V[f[0]][d]);
        push(l[0], l[1], l[2]);
      }
  for (int i = 1; i < p; ++i)
    for (int j = 1; j < p; ++j)
      for (int k = 1; k < p; ++k) push(i, j, k);
  return L;
}

// 1-D Lagrange polynomial l_i on nodes r, value and derivative at t.
inline void lagrange_1d(const std::vector<double>& r, int i, double t, double& v, double& dv) {
  v = 1.0;
  dv = 0.0;
  for (int m = 0; m < (int)r.size(); ++m) {
    if (m == i) continue;
    double f = (t - r[m]) / (r[i] - r[m]);
    dv = dv * f + v / (r[i] - r[m]);
    v *= f;
  }
}

// Reference basis values [nq][nn] and gradients [nq][nn][tdim] at the points of Q.
inline bool tabulate(int ct, int p, const Quadrature& Q, std::vector<double>& val, std::vector<double>& grad) {
  int td = cell_tdim(ct), nq = Q.size(), nn = num_nodes(ct, p);
  val.assign((size_t)nq * nn, 0.0);
  grad.assign((size_t)nq * nn * td, 0.0);
  if (is_simplex(ct)) {
    // barycentric lambda_0 = 1 - sum X, lambda_k = X_{k-1}; grad lambda constant
    const int TRI_E[3][2] = {{1, 2}, {0, 2}, {0, 1}};
    const int TET_E[6][2] = {{2, 3}, {1, 3}, {1, 2}, {0, 3}, {0, 2}, {0, 1}};
    int nvx = td + 1;
    for (int q = 0; q < nq; ++q) {
      double lam[4], glam[4][3] = {{0}};
      lam[0] = 1.0;
      for (int d = 0; d < td; ++d) {
        lam[d + 1] = Q.pts[q * td + d];
        lam[0] -= lam[d + 1];
        glam[0][d] = -1.0;
        glam[d + 1][d] = 1.0;
      }
      double* v = &val[(size_t)q * nn];
      double* g = &grad[(size_t)q * nn * td];
      if (p == 1) {
        for (int a = 0; a < nvx; ++a) {
          v[a] = lam[a];
          for (int d = 0; d < td; ++d) g[a * td + d] = glam[a][d];
        }
      } else if (p == 2) {
        for (int a = 0; a < nvx; ++a) {
          v[a] = lam[a] * (2.0 * lam[a] - 1.0);
          for (int d = 0; d < td; ++d) g[a * td + d] = (4.0 * lam[a] - 1.0) * glam[a][d];
        }
        int ne = td == 2 ? 3 : 6;
        for (int e = 0; e < ne; ++e) {
          int i = td == 2 ? TRI_E[e][0] : TET_E[e][0];
          int j = td == 2 ? TRI_E[e][1] : TET_E[e][1];
          v[nvx + e] = 4.0 * lam[i] * lam[j];
          for (int d = 0; d < td; ++d) g[(nvx + e) * td + d] = 4.0 * (lam[i] * glam[j][d] + lam[j] * glam[i][d]);
        }
      } else {
        return false;
      }
    }
    return true;
  }
  std::vector<double> r = line_points(p);
  std::vector<int> L = tensor_node_lattice(ct, p);
  if ((int)L.size() != 3 * nn) return false;
  for (int q = 0; q < nq; ++q)
    for (int a = 0; a < nn; ++a) {
      double v[3] = {1, 1, 1}, dv[3] = {0, 0, 0};
      for (int d = 0; d < td; ++d) lagrange_1d(r, L[3 * a + d], Q.pts[q * td + d], v[d], dv[d]);
      val[(size_t)q * nn + a] = v[0] * v[1] * v[2];
      double* g = &grad[((size_t)q * nn + a) * td];
      if (td == 2) {
        g[0] = dv[0] * v[1];
        g[1] = v[0] * dv[1];
      } else {
        g[0] = dv[0] * v[1] * v[2];
        g[1] = v[0] * dv[1] * v[2];
        g[2] = v[0] * v[1] * dv[2];
      }
    }
  return true;
}

// 1-D matrices of a tensor element on [0, 1] with the n-point Gauss rule of make_quadrature(ct, qdeg)
// (n = (qdeg + 2) / 2 per direction), [3][p+1][p+1]: S_ij = int l_i' l_j', M_ij = int l_i l_j,
// C_ij = int l_i' l_j. On an affine (parallelepiped) cell the reference grad-grad tensor of
// nodes a = (a0, a1, a2), b factorises: Ahat_ab[j][l] = prod_d F_d with F_d = S (d = j = l),
// C[a_d][b_d] (d = j != l), C[b_d][a_d] (d = l != j), M (otherwise) -- equal to the tensor rule's
// sum (which is exact for these degrees) up to rounding.
inline void tensor_1d_mats(int p, int qdeg, std::vector<double>& out) {
  std::vector<double> x, w;
  gauss_legendre_01((qdeg + 2) / 2, x, w);
  std::vector<double> r = line_points(p);
  const int n1 = p + 1;
  out.assign(3 * n1 * n1, 0.0);
  for (size_t q = 0; q < x.size(); ++q) {
    double v[4], dv[4];
    for (int i = 0; i < n1; ++i) lagrange_1d(r, i, x[q], v[i], dv[i]);
    for (int i = 0; i < n1; ++i)
      for (int j = 0; j < n1; ++j) {
        out[0 * n1 * n1 + i * n1 + j] += w[q] * dv[i] * dv[j];
        out[1 * n1 * n1 + i * n1 + j] += w[q] * v[i] * v[j];
        out[2 * n1 * n1 + i * n1 + j] += w[q] * dv[i] * v[j];
      }
  }
}

// Everything a kernel needs about one (cell, degree, quadrature degree) combination.
struct ElementTables {
  int ct = 0, p = 0, td = 0, nn = 0, nv = 0, nq = 0, qdeg = 0;
  std::vector<double> wq;     // [nq]
  std::vector<double> phi;    // [nq][nn]
  std::vector<double> dphi;   // [nq][nn][td]
  std::vector<double> gdphi;  // [nq][nv][td]  geometry (P1 / Q1) gradients
  std::vector<double> gphi;   // [nq][nv]      geometry values
};

inline bool make_tables(int ct, int p, int qdeg, ElementTables& T) {
  if (!supported(ct, p)) return false;
  if (qdeg < 0) qdeg = estimated_qdeg(ct, p);
  Quadrature Q = make_quadrature(ct, qdeg);
  T.ct = ct;
  T.p = p;
  T.td = cell_tdim(ct);
  T.nn = num_nodes(ct, p);
  T.nv = cell_nverts(ct);
  T.nq = Q.size();
  T.qdeg = qdeg;
  T.wq = Q.wts;
  if (!tabulate(ct, p, Q, T.phi, T.dphi)) return false;
  if (!tabulate(ct, 1, Q, T.gphi, T.gdphi)) return false;
  return true;
}

}  // namespace femasm

// femasm — MI355X (gfx950) element-stiffness assembly: kernels and the C ABI (include/femasm.h).
//
// Hot path: the reference's J assembly (FEniCSx/mechanic2d/asym_elasto_damage_model.cc:847-862,
// MFEM/mechanic2d/asym_elasto_damage_model.cc:639-916): for every cell, K_e = sum_q w_q |J_q|
// B_q^T D B_q, zero bc rows/cols, add into the global matrix, set bc diagonals.
//
// Two device algorithms produce the same BSR matrix:
//  * GATHER (default). Block rows are cut into chunks whose BSR values fit in LDS. A
//    workgroup owns one chunk: it walks the node->cell adjacency of its rows, computes for
//    every (row node a, cell c, column node b) the 3x3 block K_e[a,b] in registers, adds it
//    into the LDS copy of the chunk (ds_add_f64), sets bc diagonals, then streams the chunk
//    to HBM with plain coalesced stores. Every matrix value is written exactly once; no
//    zeroing pass, no global atomics.
//  * SCATTER. One thread per (cell, a, b) block adds it into the global BSR with FP64
//    atomics after a row-local binary search — the dolfinx/PETSc ADD_VALUES shape. Measured
//    on MI355X at ~0.7 TB/s of added bytes vs ~5 TB/s for coalesced stores, so it is the
//    cross-check / generic path, not the fast path.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cfloat>
#include <cstdarg>
#include <cstdlib>
#include <cstring>
#include <cstdio>
#include <map>
#include <mutex>
#include <string>
#include <tuple>
#include <type_traits>
#include <vector>

#include "../../include/femasm.h"
#include "elements.h"

using namespace femasm;

// ------------------------------------------------------------------------------------ errors
static thread_local std::string g_err;

static int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

#define HIP_TRY(expr)                                                                          \
  do {                                                                                         \
    hipError_t e_ = (expr);                                                                    \
    if (e_ != hipSuccess) return fail(FA_E_HIP, "%s: %s (%s:%d)", #expr, hipGetErrorString(e_), \
                                      __FILE__, __LINE__);                                     \
  } while (0)

#define LAUNCH_CHECK()                                                                           \
  do {                                                                                           \
    hipError_t e_ = hipGetLastError();                                                           \
    if (e_ != hipSuccess) return fail(FA_E_HIP, "kernel launch: %s (%s:%d)", hipGetErrorString(e_), \
                                      __FILE__, __LINE__);                                       \
  } while (0)

extern "C" const char* fa_last_error(void) { return g_err.c_str(); }
extern "C" int fa_version(void) { return 100; }

// ------------------------------------------------------------------------------------ tables
// Device copy of ElementTables, cached per (device, cell, degree, qdeg). Layout of `buf`:
// wq[nq] | dphi[nq][nn][td] | gdphi[nq][nv][td] | phi[nq][nn] | gphi[nq][nv]
struct DevTables {
  int ct, p, td, nn, nv, nq, qdeg;
  const double* wq;
  const double* dphi;
  const double* gdphi;
  const double* phi;
  const double* gphi;
  const double* ahat;  // simplex only: [nn][nn][td][td] = sum_q w_q dphi_a(q) dphi_b(q)^T
  const double* t1d;   // tensor cells: 1-D matrices S, M, C [3][p+1][p+1] (tensor_1d_mats)
  const double* lat;   // tensor cells: node lattice code a0 + 8 a1 + 64 a2 per node (as doubles)
  // tensor cells: the 1-D factors of the tabulation (tabulate() in elements.h): Gauss points x[n1],
  // then the lattice-order 1-D Lagrange values v[n1][p+1] and derivatives dv[n1][p+1] at them;
  // dphi[q][a][0] = dv[qx][ax] v[qy][ay] v[qz][az] (q = (qx n1 + qy) n1 + qz), bit for bit
  const double* g1d;
  int n1q;
  int ndoubles;
  double amax;         // simplex: max |ahat| entry (bounds the blocks of the fixed-point gather)
  // simplex: ahat = N / D with small integers N (exact rational integrals), each block's GD x GD
  // integers packed in one 64-bit word (pk_word); NULL if the element's table does not pack
  const uint64_t* pk;
  double pk_scale;     // 1 / sqrt(D)
  double pk_amax;      // max |N|
};

// Packed reference-tensor block: GD x GD signed fields, entries 0..PK0-1 in the low dword at
// PKW-bit offsets, the rest in the high dword (no field straddles the dwords).
constexpr int pk_width(int gd) { return gd == 3 ? 6 : 16; }
constexpr int pk_low(int gd) { return gd == 3 ? 5 : 2; }
static bool pack_ahat(int nn, int td, const std::vector<double>& ahat, std::vector<uint64_t>& pk, double& scale,
                      double& nmax, int* denom = nullptr) {
  if (td != 2 && td != 3) return false;
  const int w = pk_width(td), lo = pk_low(td), lim = (1 << (w - 1)) - 1;
  double amax = 0.0;
  for (double v : ahat) amax = std::max(amax, std::fabs(v));
  for (int D = 1; D <= 100000; ++D) {
    bool ok = true;
    nmax = 0.0;
    // D * Ahat must be integral up to the rounding of the quadrature sums (a few ulp of the table's
    // largest entry), not merely close: a near-rational table (another rule) keeps the double table
    const double tol = 64.0 * DBL_EPSILON * std::max(1.0, amax * D);
    for (double v : ahat) {
      const double n = std::nearbyint(v * D);
      if (std::fabs(v * D - n) > tol || std::fabs(n) > lim) {
        ok = false;
        break;
      }
      nmax = std::max(nmax, std::fabs(n));
    }
    if (!ok) continue;
    pk.assign((size_t)nn * nn, 0ull);
    for (int t = 0; t < nn * nn; ++t)
      for (int e = 0; e < td * td; ++e) {
        const int64_t n = (int64_t)std::nearbyint(ahat[(size_t)t * td * td + e] * D);
        const uint64_t f = (uint64_t)n & ((1ull << w) - 1);
        pk[t] |= e < lo ? f << (w * e) : f << (32 + w * (e - lo));
      }
    scale = 1.0 / std::sqrt((double)D);
    if (denom) *denom = D;
    return true;
  }
  return false;
}

// Ahat[a][b][i][j] = sum_q w_q dphi_a(q)[i] dphi_b(q)[j] of a simplex element's rule
static void simplex_ahat(const ElementTables& T, std::vector<double>& ah, double& amax) {
  ah.clear();
  amax = 0.0;
  for (int a = 0; a < T.nn; ++a)
    for (int b = 0; b < T.nn; ++b)
      for (int i = 0; i < T.td; ++i)
        for (int j = 0; j < T.td; ++j) {
          double v = 0.0;
          for (int q = 0; q < T.nq; ++q)
            v += T.wq[q] * T.dphi[((size_t)q * T.nn + a) * T.td + i] * T.dphi[((size_t)q * T.nn + b) * T.td + j];
          ah.push_back(v);
          amax = std::max(amax, std::fabs(v));
        }
}

static std::mutex g_tab_mu;
static std::map<std::tuple<int, int, int, int>, DevTables> g_tabs;

static int get_tables(int ct, int p, int qdeg, DevTables* out) {
  int dev = 0;
  HIP_TRY(hipGetDevice(&dev));
  if (!supported(ct, p)) return fail(FA_E_UNSUPPORTED, "unsupported element: cell %d degree %d", ct, p);
  int qd = qdeg < 0 ? estimated_qdeg(ct, p) : qdeg;
  if (qd > 12) return fail(FA_E_UNSUPPORTED, "quadrature degree %d > 12", qd);
  std::lock_guard<std::mutex> lock(g_tab_mu);
  auto key = std::make_tuple(dev, ct, p, qd);
  auto it = g_tabs.find(key);
  if (it != g_tabs.end()) {
    *out = it->second;
    return FA_OK;
  }
  ElementTables T;
  if (!make_tables(ct, p, qd, T)) return fail(FA_E_UNSUPPORTED, "element tables failed for cell %d degree %d", ct, p);
  std::vector<double> h;
  h.insert(h.end(), T.wq.begin(), T.wq.end());
  h.insert(h.end(), T.dphi.begin(), T.dphi.end());
  h.insert(h.end(), T.gdphi.begin(), T.gdphi.end());
  h.insert(h.end(), T.phi.begin(), T.phi.end());
  h.insert(h.end(), T.gphi.begin(), T.gphi.end());
  // reference tensor of grad-grad products (affine simplices: G_ab = |J| Ji^T Ahat_ab Ji)
  const size_t off_ahat = h.size();
  double amax = 0.0;
  std::vector<double> ah;
  if (is_simplex(ct)) {
    simplex_ahat(T, ah, amax);
    h.insert(h.end(), ah.begin(), ah.end());
  } else if (ct == FA_QUADRILATERAL || (ct == FA_HEXAHEDRON && p == 1)) {
    // affine quadrilaterals (parallelograms) and Q1 parallelepipeds share the simplex form: one
    // Jacobian per cell, so k_gather_lin reads the same packed table (round 6); the Gauss rule
    // integrates it exactly (Q2 / Q3 hexahedra have more dofs than a record's 32 bc bits)
    double am = 0.0;
    simplex_ahat(T, ah, am);
  }
  std::vector<uint64_t> pk;
  double pk_scale = 0.0, pk_amax = 0.0;
  size_t off_pk = 0;
  if (!ah.empty() && pack_ahat(T.nn, T.td, ah, pk, pk_scale, pk_amax)) {
    off_pk = h.size();
    for (uint64_t q : pk) {
      double d;
      std::memcpy(&d, &q, 8);
      h.push_back(d);
    }
  }
  // tensor cells: 1-D matrices of the affine fast path and the node lattice codes
  size_t off_t1d = 0, off_lat = 0, off_g1d = 0;
  int n1q = 0;
  if (!is_simplex(ct)) {
    std::vector<double> t1;
    tensor_1d_mats(p, qd, t1);
    off_t1d = h.size();
    h.insert(h.end(), t1.begin(), t1.end());
    off_lat = h.size();
    std::vector<int> L = tensor_node_lattice(ct, p);
    for (int a = 0; a < T.nn; ++a) h.push_back((double)(L[3 * a] + 8 * L[3 * a + 1] + 64 * L[3 * a + 2]));
    std::vector<double> gx, gw;
    gauss_legendre_01((std::max(qd, 1) + 2) / 2, gx, gw);
    const std::vector<double> r = line_points(p);
    n1q = (int)gx.size();
    off_g1d = h.size();
    h.insert(h.end(), gx.begin(), gx.end());
    std::vector<double> v1((size_t)n1q * (p + 1)), d1((size_t)n1q * (p + 1));
    for (int q = 0; q < n1q; ++q)
      for (int i = 0; i <= p; ++i) lagrange_1d(r, i, gx[q], v1[(size_t)q * (p + 1) + i], d1[(size_t)q * (p + 1) + i]);
    h.insert(h.end(), v1.begin(), v1.end());
    h.insert(h.end(), d1.begin(), d1.end());
  }
  double* d = nullptr;
  HIP_TRY(hipMalloc(&d, h.size() * sizeof(double)));
  HIP_TRY(hipMemcpy(d, h.data(), h.size() * sizeof(double), hipMemcpyHostToDevice));
  DevTables D;
  D.ct = ct; D.p = p; D.td = T.td; D.nn = T.nn; D.nv = T.nv; D.nq = T.nq; D.qdeg = qd;
  D.wq = d;
  D.dphi = D.wq + T.nq;
  D.gdphi = D.dphi + (size_t)T.nq * T.nn * T.td;
  D.phi = D.gdphi + (size_t)T.nq * T.nv * T.td;
  D.gphi = D.phi + (size_t)T.nq * T.nn;
  D.ahat = is_simplex(ct) ? d + off_ahat : nullptr;
  D.t1d = is_simplex(ct) ? nullptr : d + off_t1d;
  D.lat = is_simplex(ct) ? nullptr : d + off_lat;
  D.g1d = is_simplex(ct) ? nullptr : d + off_g1d;
  D.n1q = n1q;
  D.ndoubles = (int)h.size();
  D.amax = amax;
  D.pk = off_pk ? reinterpret_cast<const uint64_t*>(d + off_pk) : nullptr;
  D.pk_scale = pk_scale;
  D.pk_amax = pk_amax;
  g_tabs[key] = D;
  *out = D;
  return FA_OK;
}

extern "C" int fa_element_info(int32_t cell_type, int32_t degree, int32_t qdeg, int32_t* nn, int32_t* nq) {
  if (!supported(cell_type, degree)) return fail(FA_E_UNSUPPORTED, "unsupported element: cell %d degree %d", cell_type, degree);
  int qd = qdeg < 0 ? estimated_qdeg(cell_type, degree) : qdeg;
  if (nn) *nn = num_nodes(cell_type, degree);
  if (nq) *nq = make_quadrature(cell_type, qd).size();
  return FA_OK;
}

// Host only (no device call): whether the element's reference tensor packs into the integer table the
// table gather reads (k_gather_lin: P2 / P3 simplices, affine quadrilaterals), and its denominator D
// (Ahat = N / D); 0 = not packed (the kernel then falls back to the generic gather).
extern "C" int fa_element_table_info(int32_t cell_type, int32_t degree, int32_t qdeg, int32_t* packed_denom,
                                     double* amax) {
  if (!supported(cell_type, degree)) return fail(FA_E_UNSUPPORTED, "unsupported element: cell %d degree %d", cell_type, degree);
  const int qd = qdeg < 0 ? estimated_qdeg(cell_type, degree) : qdeg;
  if (qd > 12) return fail(FA_E_UNSUPPORTED, "quadrature degree %d > 12", qd);
  int D = 0;
  double am = 0.0;
  if (is_simplex(cell_type) || cell_type == FA_QUADRILATERAL || (cell_type == FA_HEXAHEDRON && degree == 1)) {
    ElementTables T;
    if (!make_tables(cell_type, degree, qd, T)) return fail(FA_E_UNSUPPORTED, "element tables failed");
    std::vector<double> ah;
    simplex_ahat(T, ah, am);
    std::vector<uint64_t> pk;
    double sc = 0.0, nm = 0.0;
    if (!pack_ahat(T.nn, T.td, ah, pk, sc, nm, &D)) D = 0;
  }
  if (packed_denom) *packed_denom = D;
  if (amax) *amax = am;
  return FA_OK;
}

typedef double fa_dv2 __attribute__((ext_vector_type(2)));
// Store-data registers: a VALU write to a VGPR that a buffer_store_dwordx4 issued a few instructions
// earlier still reads corrupts the stored value on gfx950 (measured: the low dword of a drained value
// replaced by the next store's offset, 2 wait states after the store; the compiler inserts none or
// two). The drains therefore keep their store data live until after the next barrier.
// Outside the gathers' loops: wait for the wave's stores (their data has then been read), the
// stored values kept live until then.
__device__ __forceinline__ void store_fence() { __builtin_amdgcn_s_waitcnt(0x0F70); }  // vmcnt(0)
template <int N>
__device__ __forceinline__ void store_fence(const double (&v)[N]) {
  store_fence();
#pragma unroll
  for (int u = 0; u < N; ++u) asm volatile("" ::"v"(v[u]));
}
template <int N, int M>
__device__ __forceinline__ void store_fence(const double (&v)[N][M]) {
  store_fence();
#pragma unroll
  for (int u = 0; u < N; ++u)
#pragma unroll
    for (int w = 0; w < M; ++w) asm volatile("" ::"v"(v[u][w]));
}
// Outside the hot drains, after a >8-byte store: ONE asm statement uses the stored registers and
// holds 16 wait states, so no write to them can be scheduled before those have passed (a use in one
// statement and the nops in another would let the compiler put the write in between). The
// "memory" clobber orders it after the store. Checked on the shipped code object by
// tests/test_store_hazard.py (tools/store_hazard.py).
#define FA_GUARD_NOPS "s_nop 7\n\ts_nop 7"
#define store_guard1(a) asm volatile(FA_GUARD_NOPS ::"v"(a) : "memory")
#define store_guard2(a, b) asm volatile(FA_GUARD_NOPS ::"v"(a), "v"(b) : "memory")
#define store_guard3(a, b, c) asm volatile(FA_GUARD_NOPS ::"v"(a), "v"(b), "v"(c) : "memory")
#define store_guard4(a, b, c, d) asm volatile(FA_GUARD_NOPS ::"v"(a), "v"(b), "v"(c), "v"(d) : "memory")
template <int N>
__device__ __forceinline__ void keep_vgprs(const fa_dv2 (&v)[N], double a, double b) {
#pragma unroll
  for (int u = 0; u < N; ++u) asm volatile("" ::"v"(v[u]));
  asm volatile("" ::"v"(a), "v"(b));
}

// AMD dispatches are limited to < 2^32 work-items (a larger grid fails silently): every kernel is
// grid-stride and grids are capped at kMaxBlocks (x 256 threads < 2^32; multiple of 8 for the
// XCD-aware gather order).
static constexpr int64_t kMaxBlocks = (1 << 24) - 8;

// ------------------------------------------------------------------------------------ device math
// Kernel-side views (passed by value).
struct MeshView {
  const int32_t* cells;
  const int32_t* geom;
  const double* x;
  int64_t ncells;
  int64_t nnodes;
  int nn, nv, gd;
};

struct FormView {
  int kind;
  int ad;  // FA_ASYM_DAMAGE_AD: the damage law's tangent and stress by AD of its potential (USE_AD)
  const double* E;
  double nu;
  const double* lam;
  const double* mu;
  const double* u;
  const double* d;
  const double* f;
};

struct BsrView {
  const int64_t* indptr;
  const int32_t* indices;
  double* data;        // window base: block indptr[row_begin]
  int64_t row_begin;   // window [row_begin, row_end)
  int64_t row_end;
};

// cell_lame in two steps (a load issued early, the arithmetic later): same values bit for bit
__device__ __forceinline__ void cell_lame_load(const FormView& F, int64_t c, double& a, double& b) {
  if (F.E) {
    a = F.E[c];
    b = 0.0;
  } else {
    a = F.lam[c];
    b = F.mu[c];
  }
}
__device__ __forceinline__ void cell_lame_from(const FormView& F, double a, double b, double& lam, double& mu) {
  if (F.E) {
    const double E = a, nu = F.nu;
    mu = E / (2.0 * (1.0 + nu));
    lam = E * nu / ((1.0 + nu) * (1.0 - 2.0 * nu));
  } else {
    lam = a;
    mu = b;
  }
}
__device__ __forceinline__ void cell_lame(const FormView& F, int64_t c, double& lam, double& mu) {
  if (F.E) {
    double E = F.E[c], nu = F.nu;
    mu = E / (2.0 * (1.0 + nu));
    lam = E * nu / ((1.0 + nu) * (1.0 - 2.0 * nu));
  } else {
    lam = F.lam[c];
    mu = F.mu[c];
  }
}

// J[i][k] = sum_v x_v[i] * gdphi_v[k]; returns det, Jinv[k][i] (row-major, stride GD).
template <int GD>
__device__ __forceinline__ double jac_inv(const double (&J)[GD][GD], double (&Ji)[GD][GD]) {
  if constexpr (GD == 2) {
    double det = J[0][0] * J[1][1] - J[0][1] * J[1][0];
    double r = 1.0 / det;
    Ji[0][0] = J[1][1] * r; Ji[0][1] = -J[0][1] * r;
    Ji[1][0] = -J[1][0] * r; Ji[1][1] = J[0][0] * r;
    return det;
  } else {
    double c00 = J[1][1] * J[2][2] - J[1][2] * J[2][1];
    double c01 = J[1][2] * J[2][0] - J[1][0] * J[2][2];
    double c02 = J[1][0] * J[2][1] - J[1][1] * J[2][0];
    double det = J[0][0] * c00 + J[0][1] * c01 + J[0][2] * c02;
    double r = 1.0 / det;
    Ji[0][0] = c00 * r;
    Ji[0][1] = (J[0][2] * J[2][1] - J[0][1] * J[2][2]) * r;
    Ji[0][2] = (J[0][1] * J[1][2] - J[0][2] * J[1][1]) * r;
    Ji[1][0] = c01 * r;
    Ji[1][1] = (J[0][0] * J[2][2] - J[0][2] * J[2][0]) * r;
    Ji[1][2] = (J[0][2] * J[1][0] - J[0][0] * J[1][2]) * r;
    Ji[2][0] = c02 * r;
    Ji[2][1] = (J[0][1] * J[2][0] - J[0][0] * J[2][1]) * r;
    Ji[2][2] = (J[0][0] * J[1][1] - J[0][1] * J[1][0]) * r;
    return det;
  }
}

// Affine simplex: J columns are edge vectors from vertex 0.
template <int GD>
__device__ __forceinline__ double simplex_geometry(const MeshView& M, int64_t c, double (&Ji)[GD][GD]) {
  const int32_t* g = M.geom + c * (GD + 1);
  double x0[GD];
  double J[GD][GD];
  int v0 = g[0];
#pragma unroll
  for (int i = 0; i < GD; ++i) x0[i] = M.x[(int64_t)v0 * GD + i];
#pragma unroll
  for (int k = 0; k < GD; ++k) {
    int vk = g[k + 1];
#pragma unroll
    for (int i = 0; i < GD; ++i) J[i][k] = M.x[(int64_t)vk * GD + i] - x0[i];
  }
  return jac_inv<GD>(J, Ji);
}

// Affine tensor cell (parallelogram / parallelepiped): J columns are the edges from vertex 0 to the
// vertices at xi = e_k (basix order: vertices 1, 2 and, in 3-D, 4). Only valid where the cell is
// affine (fa_plan_gather checks every cell and sets FA_PLAN_AFFINE).
template <int GD, int NV>
__device__ __forceinline__ double affine_tensor_geometry(const MeshView& M, int64_t c, double (&Ji)[GD][GD]) {
  const int32_t* g = M.geom + c * NV;
  double x0[GD], J[GD][GD];
  const int v0 = g[0];
#pragma unroll
  for (int i = 0; i < GD; ++i) x0[i] = M.x[(int64_t)v0 * GD + i];
#pragma unroll
  for (int k = 0; k < GD; ++k) {
    const int vk = g[1 << k];
#pragma unroll
    for (int i = 0; i < GD; ++i) J[i][k] = M.x[(int64_t)vk * GD + i] - x0[i];
  }
  return jac_inv<GD>(J, Ji);
}

// Q1 geometry at quadrature point q (tables gdphi [nq][nv][GD]).
template <int GD, int NV>
__device__ __forceinline__ double tensor_geometry(const double (&xv)[NV][GD], const double* gdphi_q, double (&Ji)[GD][GD]) {
  double J[GD][GD];
#pragma unroll
  for (int i = 0; i < GD; ++i)
#pragma unroll
    for (int k = 0; k < GD; ++k) J[i][k] = 0.0;
#pragma unroll
  for (int v = 0; v < NV; ++v)
#pragma unroll
    for (int i = 0; i < GD; ++i)
#pragma unroll
      for (int k = 0; k < GD; ++k) J[i][k] += xv[v][i] * gdphi_q[v * GD + k];
  return jac_inv<GD>(J, Ji);
}

// geometry at quadrature point q of cell c: Jinv and |det J| (affine simplex: constant)
template <int GD, int NV>
__device__ __forceinline__ double cell_geometry_q(const MeshView& M, int64_t c, const double* gdphi_q,
                                                  double (&Ji)[GD][GD]) {
  if constexpr (NV == GD + 1) {
    return fabs(simplex_geometry<GD>(M, c, Ji));
  } else {
    double xv[NV][GD];
    const int32_t* gv = M.geom + c * NV;
#pragma unroll
    for (int v = 0; v < NV; ++v)
#pragma unroll
      for (int i = 0; i < GD; ++i) xv[v][i] = M.x[(int64_t)gv[v] * GD + i];
    return fabs(tensor_geometry<GD, NV>(xv, gdphi_q, Ji));
  }
}

// physical gradient g[d] = sum_k dphi[k] Ji[k][d]
template <int GD>
__device__ __forceinline__ void phys_grad(const double* dphi, const double (&Ji)[GD][GD], double (&g)[GD]) {
#pragma unroll
  for (int d = 0; d < GD; ++d) {
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < GD; ++k) s += dphi[k] * Ji[k][d];
    g[d] = s;
  }
}

// Linear-elasticity block from G = sum_q w|J| g_a g_b^T:
// K_ab[i][j] = lam G[i][j] + mu G[j][i] + mu tr(G) delta_ij
template <int GD>
__device__ __forceinline__ void lin_block(const double (&G)[GD][GD], double lam, double mu, double (&K)[GD][GD]) {
  // K = lam G + mu G^T + mu tr(G) I, written without "+ 0.0" terms (the compiler must keep those)
  double tr = G[0][0];
#pragma unroll
  for (int i = 1; i < GD; ++i) tr += G[i][i];
  const double mtr = mu * tr, lm = lam + mu;
#pragma unroll
  for (int i = 0; i < GD; ++i)
#pragma unroll
    for (int j = 0; j < GD; ++j) K[i][j] = (i == j) ? fma(lm, G[i][i], mtr) : fma(mu, G[j][i], lam * G[i][j]);
}

// ------------------------------------------------------------------------------------ AD: dual numbers
// Forward-mode dual numbers, nested for second derivatives: the Hessian of a potential psi(F) is
// taken entry by entry over the upper triangle, seeding x_i in the inner and x_j in the outer
// level (the forward-over-forward pattern of the reference's MFEM AD,
// MFEM/mechanic2d/autodiff/admfem.hpp:672-700: n(n+1)/2 evaluations; here n = gdim^2).
template <class T>
struct Dual {
  T v, d;
};
template <class T>
__device__ __forceinline__ Dual<T> operator+(const Dual<T>& a, const Dual<T>& b) { return {a.v + b.v, a.d + b.d}; }
template <class T>
__device__ __forceinline__ Dual<T> operator-(const Dual<T>& a, const Dual<T>& b) { return {a.v - b.v, a.d - b.d}; }
template <class T>
__device__ __forceinline__ Dual<T> operator*(const Dual<T>& a, const Dual<T>& b) { return {a.v * b.v, a.d * b.v + a.v * b.d}; }
template <class T>
__device__ __forceinline__ Dual<T> operator*(double s, const Dual<T>& a) { return {s * a.v, s * a.d}; }
template <class T>
__device__ __forceinline__ Dual<T> operator+(const Dual<T>& a, double s) { return {a.v + s, a.d}; }
__device__ __forceinline__ double ad_inv(double x) { return 1.0 / x; }
template <class T>
__device__ __forceinline__ Dual<T> ad_inv(const Dual<T>& a) {
  T r = ad_inv(a.v);
  return {r, (-1.0) * (a.d * r * r)};
}
__device__ __forceinline__ double ad_log(double x) { return log(x); }
template <class T>
__device__ __forceinline__ Dual<T> ad_log(const Dual<T>& a) { return {ad_log(a.v), a.d * ad_inv(a.v)}; }

__device__ __forceinline__ double ad_sqrt(double x) { return sqrt(x); }
template <class T>
__device__ __forceinline__ Dual<T> ad_sqrt(const Dual<T>& a) {
  T r = ad_sqrt(a.v);
  return {r, 0.5 * (a.d * ad_inv(r))};
}
__device__ __forceinline__ double ad_val(double x) { return x; }
template <class T>
__device__ __forceinline__ double ad_val(const Dual<T>& a) { return ad_val(a.v); }

// The reference's asymmetric damage potential psi(strain; lam, mu, d) (MFEM/mechanic2d/
// asym_elasto_damage_model.cc:100-155, the functor its USE_AD build differentiates), strain state
// (e11, e21, e12, e22): lam/2 I1^2 (1 - alpha d) + mu sum_k (1 - alpha_k d) ev_k^2 with the
// principal strains ev_k and alpha = [I1 >= 0], alpha_k = [ev_k >= 0] (branch tests on the primal
// values, as the AD types compare); the "null tensor" branch is the linear potential scaled by 1 - d.
template <class T>
__device__ __forceinline__ T damage_potential(const T (&e)[4], double l, double m, double d) {
  const double limit = 1.e-12, mlimit = -1.e-12;
  const T I1 = e[0] + e[3];
  const T I2 = e[1] * e[2] - e[0] * e[3];
  const double i1 = ad_val(I1), i2 = ad_val(I2);
  if (i1 > limit || i2 > limit || i1 < mlimit || i2 < mlimit) {
    const T delta = I1 * I1 + 4.0 * I2;
    const T r = ad_sqrt(delta);
    const T ev1 = 0.5 * (I1 + r), ev2 = 0.5 * (I1 - r);
    const double alpha1 = ad_val(ev1) >= 0.0 ? 1.0 : 0.0, alpha2 = ad_val(ev2) >= 0.0 ? 1.0 : 0.0;
    const double alpha = (ad_val(ev1) + ad_val(ev2)) >= 0.0 ? 1.0 : 0.0;
    return (0.5 * (1.0 - alpha * d) * l) * (I1 * I1) +
           m * ((1.0 - alpha1 * d) * (ev1 * ev1) + (1.0 - alpha2 * d) * (ev2 * ev2));
  }
  return (1.0 - d) * ((0.5 * l) * (I1 * I1) + m * (e[0] * e[0] + e[3] * e[3] + e[1] * e[1] + e[2] * e[2]));
}

// USE_AD tangent (MFEM/mechanic2d/asym_elasto_damage_model.cc:735-765): for d > 0 (limited to
// 1 - 1e-12) the Hessian of damage_potential over the 4 strain components by forward-over-forward
// AD, upper triangle (admfem.hpp:672-700: n(n+1)/2 = 10 passes), reordered to Voigt (xx, yy, xy):
// hook(i, j) = hess(i + 2 (i % 2), j + 2 (j % 2)), hook(2, 2) = (hess(2, 2) + hess(1, 2)) / 2
// (:761-763). d = 0 keeps the linear branch (:873-881), as the reference never differentiates there.
__device__ __noinline__ void damage_hook_ad(double s00, double s11, double s01, double l, double m, double d,
                                            double (&H)[3][3]) {
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) H[i][j] = 0.0;
  if (!(d > 0.0)) {
    H[0][0] = H[1][1] = 2.0 * m + l;
    H[0][1] = H[1][0] = l;
    H[2][2] = m;
    return;
  }
  d = fmin(d, 1.0 - 1.e-12);
  const double st[4] = {s00, s01, s01, s11};  // column-major strain: e11, e21, e12, e22
  using DD = Dual<Dual<double>>;
  double hs[4][4];
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j <= i; ++j) {
      DD x[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) x[k] = DD{{st[k], k == i ? 1.0 : 0.0}, {k == j ? 1.0 : 0.0, 0.0}};
      const double h = damage_potential<DD>(x, l, m, d).d.d;
      hs[i][j] = h;
      hs[j][i] = h;
    }
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) H[i][j] = hs[i + 2 * (i % 2)][j + 2 * (j % 2)];
  H[2][2] = 0.5 * (H[2][2] + hs[1][2]);
}

// USE_AD stress (asym_stress, :158-204): for d > 0 the gradient of damage_potential with the Lame
// parameters scaled by w (4 forward-mode passes), sig = [[g_e11, g_e12], [g_e21, g_e22]]; d = 0 the
// linear stress.
__device__ __noinline__ void damage_stress_ad(double s00, double s11, double s01, double l, double m, double d,
                                              double w, double (&sig)[2][2]) {
  if (!(d > 0.0)) {
    const double m2plw = w * (2.0 * m + l), lw = l * w;
    const double a = m2plw * s00 + lw * s11, b = m2plw * s11 + lw * s00, c = w * m * (s01 + s01);
    sig[0][0] = a;
    sig[1][1] = b;
    sig[0][1] = sig[1][0] = c;
    store_guard3(a, b, c);
    return;
  }
  const double st[4] = {s00, s01, s01, s11};
  using D1 = Dual<double>;
  double g[4];
  for (int i = 0; i < 4; ++i) {
    D1 x[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) x[k] = D1{st[k], k == i ? 1.0 : 0.0};
    g[i] = damage_potential<D1>(x, l * w, m * w, d).d;
  }
  sig[0][0] = g[0];
  sig[1][0] = g[1];
  sig[0][1] = g[2];
  sig[1][1] = g[3];
  store_guard4(g[0], g[1], g[2], g[3]);
}

// Reference damage-law tangent "hook" (Voigt xx, yy, xy-engineering), restated from MFEM
// damIntegrator::AssembleElementGrad (MFEM/mechanic2d/asym_elasto_damage_model.cc:728-881).
__device__ __forceinline__ void damage_hook(double s00, double s11, double s01, double l, double m, double d,
                                            double (&H)[3][3]) {
  const double limit = 1.e-12, mlimit = -1.e-12;
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) H[i][j] = 0.0;
  if (d > 0.0) {
    d = fmin(d, 1.0 - limit);
    double I1 = s00 + s11;
    double I2 = s01 * s01 - s00 * s11;
    if (I1 > limit || I2 > limit || I1 < mlimit || I2 < mlimit) {
      double delta = I1 * I1 + 4.0 * I2;
      double r = sqrt(fmax(0.0, delta));
      double e1 = 0.5 * (I1 + r), e2 = 0.5 * (I1 - r);
      double cs, sn;
      if (r < limit) {
        double sg = (2.0 * s01 / (s00 - s11)) > 0.0 ? 1.0 : -1.0;
        cs = sg * 0.70710678118654752440;  // sqrt(2)/2
        sn = cs;
      } else {
        cs = (s00 - s11) / r;
        sn = 2.0 * s01 / r;
      }
      double a1 = e1 >= 0.0 ? 1.0 : 0.0, a2 = e2 >= 0.0 ? 1.0 : 0.0, a = I1 >= 0.0 ? 1.0 : 0.0;
      double fac = 2.0 * m, gam = 0.5 * l / m;
      double c1 = 1.0 - a1 * d, c2 = 1.0 - a2 * d, c3 = 1.0 - a * d;
      double P00 = fac * (c1 + gam * c3), P01 = fac * gam * c3, P11 = fac * (c2 + gam * c3);
      double De[2][3] = {{0.5 * (1.0 + cs), 0.5 * (1.0 - cs), 0.5 * sn}, {0.5 * (1.0 - cs), 0.5 * (1.0 + cs), -0.5 * sn}};
      double cos2 = cs * cs, sin2 = sn * sn, sc = sn * cs, hm = 0.5 * m;
      double Mm[3][3] = {{hm * (1.0 - cos2), hm * (-1.0 + cos2), -hm * sc},
                         {hm * (-1.0 + cos2), hm * (1.0 - cos2), hm * sc},
                         {-hm * sc, hm * sc, hm * (1.0 - sin2)}};
      double q = (r >= limit) ? (I1 / r * (c1 - c2) + (c1 + c2)) : (c1 + c2);
#pragma unroll
      for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          double t0 = P00 * De[0][j] + P01 * De[1][j];
          double t1 = P01 * De[0][j] + P11 * De[1][j];
          H[i][j] = De[0][i] * t0 + De[1][i] * t1 + q * Mm[i][j];
        }
    } else {
      double md = (1.0 - d) * m, ld = (1.0 - d) * l;
      H[0][0] = H[1][1] = 2.0 * md + ld;
      H[0][1] = H[1][0] = ld;
      H[2][2] = md;
    }
  } else {
    H[0][0] = H[1][1] = 2.0 * m + l;
    H[0][1] = H[1][0] = l;
    H[2][2] = m;
  }
}

// Damage-law P1-triangle setup for cell c: physical gradients g[3][2], weight w = |J|/2 and
// the hook at the single quadrature point (`dxx` degree 1, FEniCSx/mechanic2d/asym_ufl.py:78).
__device__ __forceinline__ void damage_cell(const MeshView& M, const FormView& F, int64_t c, double (&g)[3][2],
                                            double& w, double (&H)[3][3]) {
  double Ji[2][2];
  double det = simplex_geometry<2>(M, c, Ji);
  w = 0.5 * fabs(det);
  const double ref[3][2] = {{-1.0, -1.0}, {1.0, 0.0}, {0.0, 1.0}};
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    double gg[2];
    phys_grad<2>(ref[a], Ji, gg);
    g[a][0] = gg[0];
    g[a][1] = gg[1];
  }
  double lam, mu;
  cell_lame(F, c, lam, mu);
  const int32_t* nd = M.cells + c * 3;
  double gr[2][2] = {{0.0, 0.0}, {0.0, 0.0}};
  double dq = 0.0;
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    int64_t n = nd[a];
    double u0 = F.u ? F.u[n * 2 + 0] : 0.0, u1 = F.u ? F.u[n * 2 + 1] : 0.0;
    gr[0][0] += u0 * g[a][0]; gr[0][1] += u0 * g[a][1];
    gr[1][0] += u1 * g[a][0]; gr[1][1] += u1 * g[a][1];
    if (F.d) dq += F.d[n];
  }
  dq *= (1.0 / 3.0);
  if (F.ad) damage_hook_ad(gr[0][0], gr[1][1], 0.5 * (gr[0][1] + gr[1][0]), lam, mu, dq, H);
  else damage_hook(gr[0][0], gr[1][1], 0.5 * (gr[0][1] + gr[1][0]), lam, mu, dq, H);
}

// K_ab = w B_a^T H B_b with B_a = [[gx,0],[0,gy],[gy,gx]] (MFEM USE_B, :699-704, :885-887)
__device__ __forceinline__ void damage_block(const double (&ga)[2], const double (&gb)[2], double w,
                                             const double (&H)[3][3], double (&K)[2][2]) {
  double Ba[3][2] = {{ga[0], 0.0}, {0.0, ga[1]}, {ga[1], ga[0]}};
  double Bb[3][2] = {{gb[0], 0.0}, {0.0, gb[1]}, {gb[1], gb[0]}};
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      double s = 0.0;
#pragma unroll
      for (int k = 0; k < 3; ++k)
#pragma unroll
        for (int l = 0; l < 3; ++l) s += Ba[k][i] * H[k][l] * Bb[l][j];
      K[i][j] = w * s;
    }
}

__device__ __forceinline__ int64_t find_slot(const int64_t* indptr, const int32_t* indices, int64_t row, int32_t col) {
  int64_t lo = indptr[row], hi = indptr[row + 1] - 1;
  while (lo <= hi) {
    int64_t mid = (lo + hi) >> 1;
    int32_t cm = indices[mid];
    if (cm == col) return mid;
    if (cm < col) lo = mid + 1;
    else hi = mid - 1;
  }
  return -1;
}

// Compressible neo-Hookean potential psi(F) = mu/2 (I_C - 3) - mu ln J + lam/2 (ln J)^2,
// F = I + grad u (2-D: plane strain, F33 = 1, so I_C - 3 = F:F - 2).
template <int GD, class T>
__device__ __forceinline__ T neo_psi(const T (&F)[GD * GD], double lam, double mu) {
  T J, ff = F[0] * F[0];
#pragma unroll
  for (int k = 1; k < GD * GD; ++k) ff = ff + F[k] * F[k];
  if constexpr (GD == 2) {
    J = F[0] * F[3] - F[1] * F[2];
  } else {
    J = F[0] * (F[4] * F[8] - F[5] * F[7]) - F[1] * (F[3] * F[8] - F[5] * F[6]) + F[2] * (F[3] * F[7] - F[4] * F[6]);
  }
  T lnJ = ad_log(J);
  return (0.5 * mu) * (ff + (-(double)GD)) - mu * lnJ + (0.5 * lam) * (lnJ * lnJ);
}

// A[(iJ)(kL)] = d^2 psi / dF_iJ dF_kL by forward-over-forward AD (upper triangle, symmetric fill).
template <int GD>
__device__ void neo_tangent_ad(const double (&F)[GD * GD], double lam, double mu, double* __restrict__ A) {
  constexpr int N = GD * GD;
  using DD = Dual<Dual<double>>;
  for (int i = 0; i < N; ++i)
    for (int j = i; j < N; ++j) {
      DD x[N];
#pragma unroll
      for (int m = 0; m < N; ++m) x[m] = DD{{F[m], m == i ? 1.0 : 0.0}, {m == j ? 1.0 : 0.0, 0.0}};
      DD r = neo_psi<GD, DD>(x, lam, mu);
      A[i * N + j] = r.d.d;
      A[j * N + i] = r.d.d;
    }
}

// P[iJ] = d psi / dF_iJ (first Piola stress) by forward-mode AD: the residual of the same potential.
template <int GD>
__device__ void neo_stress_ad(const double (&F)[GD * GD], double lam, double mu, double (&P)[GD * GD]) {
  constexpr int N = GD * GD;
  using D1 = Dual<double>;
  for (int i = 0; i < N; ++i) {
    D1 x[N];
#pragma unroll
    for (int m = 0; m < N; ++m) x[m] = D1{F[m], m == i ? 1.0 : 0.0};
    P[i] = neo_psi<GD, D1>(x, lam, mu).d;
  }
}

// The same potential in its invariants, W(I1, J) = mu/2 (I1 - 3) - mu ln J + lam/2 (ln J)^2 with
// I1 = F:F (+ 1 in 2-D plane strain), psi(F) = W(I1(F), J(F)).
template <class T>
__device__ __forceinline__ T neo_energy(const T& I1, const T& J, double lam, double mu) {
  const T lnJ = ad_log(J);
  return (0.5 * mu) * (I1 + (-3.0)) - mu * lnJ + (0.5 * lam) * (lnJ * lnJ);
}

// Tangent coefficients by forward-over-forward AD of W(I1, J) (three hyper-dual passes over the two
// invariants, seeds unrolled): with C = cof F = dJ/dF and dI1/dF = 2F,
//   d2psi/dF_iJ dF_kL = 4 W_11 F_iJ F_kL + 2 W_1J (F_iJ C_kL + C_iJ F_kL) + W_JJ C_iJ C_kL
//                       + 2 W_1 d_ik d_JL + W_J (C_iJ C_kL - C_iL C_kJ) / J,
// so a block of the element matrix needs F, C and co = {4 W_11, 2 W_1J, W_JJ + W_J / J, W_J / J, 2 W_1}.
__device__ __forceinline__ void neo_energy_coeffs(double I1, double J, double lam, double mu, double (&co)[5]) {
  using DD = Dual<Dual<double>>;
  double W[2][2], G[2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = a; b < 2; ++b) {
      const DD x1{{I1, a == 0 ? 1.0 : 0.0}, {b == 0 ? 1.0 : 0.0, 0.0}};
      const DD xJ{{J, a == 1 ? 1.0 : 0.0}, {b == 1 ? 1.0 : 0.0, 0.0}};
      const DD r = neo_energy(x1, xJ, lam, mu);
      W[a][b] = W[b][a] = r.d.d;
      G[a] = r.v.d;
    }
  co[0] = 4.0 * W[0][0];
  co[1] = 2.0 * W[0][1];
  co[2] = W[1][1] + G[1] / J;
  co[3] = G[1] / J;
  co[4] = 2.0 * G[0];
}

// cofactor matrix C = dJ/dF of a row-major F (F[i * GD + J])
template <int GD>
__device__ __forceinline__ void cofactor(const double (&F)[GD * GD], double (&C)[GD][GD]) {
  if constexpr (GD == 2) {
    C[0][0] = F[3]; C[0][1] = -F[2]; C[1][0] = -F[1]; C[1][1] = F[0];
  } else {
    C[0][0] = F[4] * F[8] - F[5] * F[7]; C[0][1] = F[5] * F[6] - F[3] * F[8]; C[0][2] = F[3] * F[7] - F[4] * F[6];
    C[1][0] = F[2] * F[7] - F[1] * F[8]; C[1][1] = F[0] * F[8] - F[2] * F[6]; C[1][2] = F[1] * F[6] - F[0] * F[7];
    C[2][0] = F[1] * F[5] - F[2] * F[4]; C[2][1] = F[2] * F[3] - F[0] * F[5]; C[2][2] = F[0] * F[4] - F[1] * F[3];
  }
}

// F at a quadrature point from the cell's nodal displacements and physical gradients.
template <int GD>
__device__ __forceinline__ void deformation_gradient(const double* __restrict__ u, const int32_t* cn, int nn,
                                                     const double* dphi_q, const double (&Ji)[GD][GD],
                                                     double (&F)[GD * GD]) {
#pragma unroll
  for (int i = 0; i < GD; ++i)
#pragma unroll
    for (int k = 0; k < GD; ++k) F[i * GD + k] = (i == k) ? 1.0 : 0.0;
  for (int b = 0; b < nn; ++b) {
    double gb[GD];
    phys_grad<GD>(dphi_q + b * GD, Ji, gb);
    const int64_t n = cn[b];
#pragma unroll
    for (int i = 0; i < GD; ++i) {
      const double ui = u[n * GD + i];
#pragma unroll
      for (int k = 0; k < GD; ++k) F[i * GD + k] += ui * gb[k];
    }
  }
}

// K_ab[i][k] += w sum_{J,L} ga[J] A[(iJ)(kL)] gb[L]
template <int GD>
__device__ __forceinline__ void neo_block_add(const double* A, const double (&ga)[GD], const double (&gb)[GD], double w,
                                              double (&K)[GD][GD]) {
  constexpr int N = GD * GD;
#pragma unroll
  for (int i = 0; i < GD; ++i)
#pragma unroll
    for (int k = 0; k < GD; ++k) {
      double sacc = 0.0;
#pragma unroll
      for (int J = 0; J < GD; ++J) {
        double t = 0.0;
#pragma unroll
        for (int L = 0; L < GD; ++L) t += A[(i * GD + J) * N + k * GD + L] * gb[L];
        sacc += ga[J] * t;
      }
      K[i][k] += w * sacc;
    }
}

// ------------------------------------------------------------------------------------ generic per-block kernel
// One thread per (cell, a, b). MODE 0: write the cell matrix Ae[c][a*bs+i][b*bs+j].
// MODE 1: FP64-atomic add into BSR (bc rows/cols skipped); error flag on a missing slot.
template <int GD, int NV, int MODE>
__global__ __launch_bounds__(256) void k_cell_blocks(MeshView M, FormView F, DevTables T, int64_t c0, int64_t ncells,
                                                   double* __restrict__ Ae, BsrView A, const int8_t* __restrict__ bc,
                                                   int* __restrict__ err) {
  const int nn = T.nn;
  const int64_t per = (int64_t)nn * nn;
  const int64_t total = ncells * per;
  for (int64_t it = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; it < total; it += (int64_t)gridDim.x * blockDim.x) {
    int64_t c = c0 + it / per;
    int ab = (int)(it % per);
    int a = ab / nn, b = ab % nn;
    double K[GD][GD];
    if (F.kind == FA_ASYM_DAMAGE) {
      if constexpr (GD == 2) {
        double g[3][2], w, H[3][3];
        damage_cell(M, F, c, g, w, H);
        double ga[2] = {g[a][0], g[a][1]}, gb[2] = {g[b][0], g[b][1]};
        damage_block(ga, gb, w, H, K);
      }
    } else if (F.kind == FA_NEO_HOOKEAN) {
      double lam, mu;
      cell_lame(F, c, lam, mu);
#pragma unroll
      for (int i = 0; i < GD; ++i)
#pragma unroll
        for (int j = 0; j < GD; ++j) K[i][j] = 0.0;
      const int32_t* cn = M.cells + c * nn;
      for (int q = 0; q < T.nq; ++q) {
        double Ji[GD][GD];
        const double wd = T.wq[q] * cell_geometry_q<GD, NV>(M, c, T.gdphi + (size_t)q * NV * GD, Ji);
        double Fq[GD * GD], A[GD * GD * GD * GD];
        deformation_gradient<GD>(F.u, cn, nn, T.dphi + (size_t)q * nn * GD, Ji, Fq);
        neo_tangent_ad<GD>(Fq, lam, mu, A);
        double ga[GD], gb[GD];
        phys_grad<GD>(T.dphi + ((size_t)q * nn + a) * GD, Ji, ga);
        phys_grad<GD>(T.dphi + ((size_t)q * nn + b) * GD, Ji, gb);
        neo_block_add<GD>(A, ga, gb, wd, K);
      }
    } else {
      double lam, mu;
      cell_lame(F, c, lam, mu);
      double G[GD][GD];
#pragma unroll
      for (int i = 0; i < GD; ++i)
#pragma unroll
        for (int j = 0; j < GD; ++j) G[i][j] = 0.0;
      double xv[NV][GD];
      const bool simp = (NV == GD + 1);
      double Ji[GD][GD];
      double det = 0.0;
      if (simp) {
        det = simplex_geometry<GD>(M, c, Ji);
      } else {
        const int32_t* gv = M.geom + c * NV;
#pragma unroll
        for (int v = 0; v < NV; ++v)
#pragma unroll
          for (int i = 0; i < GD; ++i) xv[v][i] = M.x[(int64_t)gv[v] * GD + i];
      }
      for (int q = 0; q < T.nq; ++q) {
        if (!simp) det = tensor_geometry<GD, NV>(xv, T.gdphi + (size_t)q * NV * GD, Ji);
        double ga[GD], gb[GD];
        phys_grad<GD>(T.dphi + ((size_t)q * nn + a) * GD, Ji, ga);
        phys_grad<GD>(T.dphi + ((size_t)q * nn + b) * GD, Ji, gb);
        double w = T.wq[q] * fabs(det);
#pragma unroll
        for (int i = 0; i < GD; ++i)
#pragma unroll
          for (int j = 0; j < GD; ++j) G[i][j] += w * ga[i] * gb[j];
      }
      lin_block<GD>(G, lam, mu, K);
    }
    if (MODE == 0) {
      const int nd = nn * GD;
      double* out = Ae + (it / per) * (int64_t)nd * nd;
#pragma unroll
      for (int i = 0; i < GD; ++i)
#pragma unroll
        for (int j = 0; j < GD; ++j) out[(a * GD + i) * nd + b * GD + j] = K[i][j];
      store_fence(K);
    } else {
      int64_t na = M.cells[c * nn + a], nb = M.cells[c * nn + b];
      if (na < A.row_begin || na >= A.row_end) continue;
      int64_t s = find_slot(A.indptr, A.indices, na, (int32_t)nb);
      if (s < 0) {
        atomicOr(err, 1);
        continue;
      }
      double* dst = A.data + (s - A.indptr[A.row_begin]) * GD * GD;
#pragma unroll
      for (int i = 0; i < GD; ++i) {
        if (bc && bc[na * GD + i]) continue;
#pragma unroll
        for (int j = 0; j < GD; ++j) {
          if (bc && bc[nb * GD + j]) continue;
          unsafeAtomicAdd(dst + i * GD + j, K[i][j]);
        }
      }
    }
  }
}

// zero the values of the row window (bounds read on the device: no host sync)
__global__ void k_zero_window(BsrView A, int bs2) {
  const int64_t n = (A.indptr[A.row_end] - A.indptr[A.row_begin]) * bs2;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    A.data[i] = 0.0;
}

// ------------------------------------------------------------------------------------ hexahedra: MFMA
// Q1/Q2/Q3 hexahedra, linear elasticity, any trilinear geometry. One 256-thread workgroup per cell.
// With Phi_i[q][a] = sqrt(w_q |J_q|) d_i phi_a(x_q) (physical gradients), the cell's
// grad-grad products are nine small GEMMs  M_ik = Phi_i Phi_k^T  (NN x NN, inner dim = quadrature
// points), a genuine per-cell contraction that runs on v_mfma_f64_16x16x4_f64; the elasticity
// block is then register-local: K_ab[i][k] = lam M_ik[a][b] + mu M_ki[a][b] + mu d_ik tr M[a][b].
// Each lane ends with complete 3x3 blocks (4 (a,b) pairs per 16x16 tile), which MODE 0 writes to
// Ae and MODE 1 adds into the global BSR with FP64 atomics (dolfinx ADD_VALUES semantics).
typedef double fa_d4 __attribute__((ext_vector_type(4)));

// tiles per wave of k_hex_mfma: Q3 (16 tiles) runs 8 waves of 2 tiles, whose 18 accumulators fit
// the 256 VGPRs of 2 waves / SIMD (16 waves of one tile were capped at 128 VGPRs and spilled 35)
__host__ __device__ constexpr int hex_tpw(int nn) { return ((nn + 15) / 16) * ((nn + 15) / 16) >= 16 ? 2 : 1; }
__host__ __device__ constexpr int hex_threads(int nn) { return 64 * ((nn + 15) / 16) * ((nn + 15) / 16) / hex_tpw(nn); }
// every (a, b) tile is computed (the upper triangle with transposed stores measured slower on config
// Dmfma: 38.5 vs 27.5 ms, 5-wave workgroups at 2 waves / SIMD leave 3 of a CU's 8 wave slots idle)
__host__ __device__ constexpr int hex_ntiles(int nn, int mode) { return ((nn + 15) / 16) * ((nn + 15) / 16); }
__host__ __device__ constexpr int hex_threads_m(int nn, int mode) {
  return 64 * ((hex_ntiles(nn, mode) + hex_tpw(nn) - 1) / hex_tpw(nn));
}

template <int NN, int NQ, int MODE>
__global__ __launch_bounds__(hex_threads_m(NN, MODE)) void k_hex_mfma(
    MeshView M, FormView F, DevTables T, int64_t c0, int64_t ncells, double* __restrict__ Ae, BsrView A,
    const int8_t* __restrict__ bc, int* __restrict__ err) {
  constexpr int NT = (NN + 15) / 16;  // 16-row tiles per side; TPW (a, b) tiles per wave
  constexpr int NTL = hex_ntiles(NN, MODE);  // tiles computed
  constexpr int TPW = hex_tpw(NN), NWAVE = (NTL + TPW - 1) / TPW;
  constexpr int NTHR = hex_threads_m(NN, MODE);
  // tile t -> (ta, tb): row-major over the grid
  auto tile_of = [](int t, int& ta, int& tb) {
    ta = t / NT;
    tb = t % NT;
  };
  // row stride: +8 doubles puts the 4 rows q0..q0+3 a ds_read_b64 of the MFMA loop reads on 2 banks
  // each (2 passes, the minimum for 512 B); round 2's +16 left no room for the staging below
  constexpr int NNP = NT * 16 + 8;
  constexpr int QMAX = (NQ + 3) & ~3;
  constexpr int P1 = NN == 8 ? 2 : NN == 27 ? 3 : 4;  // nodes and Gauss points per direction
  constexpr int G1 = NQ == 8 ? 2 : NQ == 27 ? 3 : 4;
  static_assert(P1 * P1 * P1 == NN && G1 * G1 * G1 == NQ, "tensor element with a tensor Gauss rule");
  __shared__ double phi[3][QMAX][NNP];
  __shared__ double sJ[QMAX][10];  // Ji (9) + sqrt(w |J|)
  __shared__ uint32_t s_bcn[2][NN]; // MODE 2: byte i = dof i of the node constrained (two cells)
  // round 5: the tables of the per-cell phase (Gauss points, 1-D factors of the basis gradients,
  // weights, node lattice codes) and the cell's vertices sit in LDS, so the phase before the MFMA
  // loop issues no global load: a load there waited (vmcnt) for the previous cell's 295 KB of block
  // stores, which serialised the stores with the next cell (Dmfma: stores ~ MFMA ~ 15 us per cell)
  __shared__ double s_gx[G1], s_v1[G1][P1], s_d1[G1][P1], s_wq[NQ];
  __shared__ int s_lat[NN];
  __shared__ double s_xv[24];      // vertex v, coordinate i at 3 v + i
  __shared__ double s_st[MODE == 2 ? NWAVE : 1][64 * 9];  // MODE 2: each wave's block staging
  static_assert(NTL % TPW == 0, "whole waves of tiles");
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nq = NQ, nqp = QMAX;
  for (int t = tid; t < NQ; t += NTHR) s_wq[t] = T.wq[t];
  for (int t = tid; t < NN; t += NTHR) s_lat[t] = (int)T.lat[t];
  for (int t = tid; t < G1; t += NTHR) s_gx[t] = T.g1d[t];
  for (int t = tid; t < G1 * P1; t += NTHR) {
    s_v1[t / P1][t % P1] = T.g1d[G1 + t];
    s_d1[t / P1][t % P1] = T.g1d[G1 + G1 * P1 + t];
  }
  // The next cell's inputs are loaded one cell ahead, their indices two cells ahead: lane tid < 24
  // holds vertex tid / 3's coordinate tid % 3, lane tid < 3 NN the bc byte of dof tid % 3 of node
  // tid / 3 (MODE 2; one byte per lane: adjacent byte loads are merged and split at once, which
  // waits), every lane the cell's material values. Issued after the pre-MFMA phase, consumed after
  // the MFMA loop.
  const bool bcb = MODE == 2 && bc != nullptr;
  auto load_ids = [&](int64_t cc, int32_t& gv, int32_t& nv) {
    if (cc < ncells) {
      if (tid < 24) gv = M.geom[(c0 + cc) * 8 + tid / 3];
      if (bcb && tid < 3 * NN) nv = M.cells[(c0 + cc) * NN + tid / 3];
    }
  };
  auto load_data = [&](int64_t cc, int32_t gv, int32_t nv, double& xval, int& bb, double& la, double& lb) {
    if (cc < ncells) {
      if (tid < 24) xval = M.x[(int64_t)gv * 3 + tid % 3];
      if (bcb && tid < 3 * NN) bb = bc[(int64_t)nv * 3 + tid % 3];
      cell_lame_load(F, c0 + cc, la, lb);
    }
  };
  uint8_t* const s_bcb = reinterpret_cast<uint8_t*>(&s_bcn[0][0]);
  auto put_bc = [&](int p, int bb) {
    if (MODE == 2 && tid < 3 * NN) s_bcb[(p * NN + tid / 3) * 4 + tid % 3] = bb ? 1 : 0;
  };
  const int64_t G = gridDim.x;
  int32_t gv0 = 0, nv0 = 0, gv1 = 0, nv1 = 0;
  double xval = 0.0, la = 0.0, lb = 0.0;
  int bits = 0;
  load_ids(blockIdx.x, gv0, nv0);
  load_ids(blockIdx.x + G, gv1, nv1);
  load_data(blockIdx.x, gv0, nv0, xval, bits, la, lb);
  if (tid < 24) s_xv[tid] = xval;
  if (MODE == 2) for (int t = tid; t < NN; t += NTHR) s_bcn[0][t] = 0u;
  if (MODE == 2) for (int t = tid; t < NN; t += NTHR) s_bcn[1][t] = 0u;
  __syncthreads();
  put_bc(0, bits);
  double lam, mu;
  cell_lame_from(F, la, lb, lam, mu);
  int par = 0;
  for (int64_t ci = blockIdx.x; ci < ncells; ci += G, par ^= 1) {
    const int64_t c = c0 + ci;
    __syncthreads();  // the previous cell's staging is read; this cell's vertices / bc bits are in LDS
    if (tid < nq) {   // geometry at quadrature point q = tid (Q1 gradients from the 1-D points)
      const int qx = tid / (G1 * G1), qy = (tid / G1) % G1, qz = tid % G1;
      const double xi[3] = {s_gx[qx], s_gx[qy], s_gx[qz]};
      double xv[8][3], gd[8 * 3];
#pragma unroll
      for (int v = 0; v < 8; ++v) {
        double f[3], df[3];
#pragma unroll
        for (int d = 0; d < 3; ++d) {
          const bool hi = (v >> d) & 1;
          f[d] = hi ? xi[d] : 1.0 - xi[d];
          df[d] = hi ? 1.0 : -1.0;
        }
        gd[v * 3 + 0] = df[0] * f[1] * f[2];
        gd[v * 3 + 1] = f[0] * df[1] * f[2];
        gd[v * 3 + 2] = f[0] * f[1] * df[2];
#pragma unroll
        for (int i = 0; i < 3; ++i) xv[v][i] = s_xv[v * 3 + i];
      }
      double Ji[3][3];
      const double det = tensor_geometry<3, 8>(xv, gd, Ji);
#pragma unroll
      for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int k = 0; k < 3; ++k) sJ[tid][i * 3 + k] = Ji[i][k];
      sJ[tid][9] = sqrt(s_wq[tid] * fabs(det));
    }
    __syncthreads();
    for (int idx = tid; idx < nqp * NT * 16; idx += NTHR) {
      const int q = idx / (NT * 16), a = idx % (NT * 16);
      double g[3] = {0.0, 0.0, 0.0};
      if (q < nq && a < NN) {
        const int qx = q / (G1 * G1), qy = (q / G1) % G1, qz = q % G1;
        const int lt = s_lat[a], ax = lt & 7, ay = (lt >> 3) & 7, az = lt >> 6;
        const double vx = s_v1[qx][ax], vy = s_v1[qy][ay], vz = s_v1[qz][az];
        const double dp[3] = {s_d1[qx][ax] * vy * vz, vx * s_d1[qy][ay] * vz, vx * vy * s_d1[qz][az]};
        const double sc = sJ[q][9];
#pragma unroll
        for (int d = 0; d < 3; ++d) g[d] = sc * (dp[0] * sJ[q][d] + dp[1] * sJ[q][3 + d] + dp[2] * sJ[q][6 + d]);
      }
#pragma unroll
      for (int i = 0; i < 3; ++i) phi[i][q][a] = g[i];
    }
    // the next cell's inputs (its indices were loaded one cell earlier), the one after's indices
    int32_t gv2 = 0, nv2 = 0;
    load_data(ci + G, gv1, nv1, xval, bits, la, lb);
    load_ids(ci + 2 * G, gv2, nv2);
    __syncthreads();
    const int32_t* cn = M.cells + c * NN;
    double lam_n = 0.0, mu_n = 0.0;
    // The wave's tiles one after the other (round 5): tile j's stores drain while tile j + 1's MFMA
    // loop runs (both tiles' accumulators at once kept the stores after every MFMA of the cell), and
    // 9 accumulators instead of 18 leave registers free
#pragma unroll
    for (int j = 0; j < TPW; ++j) {
      int ta, tb;
      tile_of(wave + j * NWAVE, ta, tb);
      fa_d4 acc[9];
#pragma unroll
      for (int m = 0; m < 9; ++m) acc[m] = fa_d4{0.0, 0.0, 0.0, 0.0};
      {
        const int kq = lane >> 4;
        const int ra = ta * 16 + (lane & 15), rb = tb * 16 + (lane & 15);
#pragma unroll 2
        for (int q0 = 0; q0 < nqp; q0 += 4) {
          double av[3], bv[3];
#pragma unroll
          for (int i = 0; i < 3; ++i) {
            av[i] = phi[i][q0 + kq][ra];  // A[a][q] = Phi_i
            bv[i] = phi[i][q0 + kq][rb];  // B[q][b] = Phi_k^T
          }
#pragma unroll
          for (int i = 0; i < 3; ++i)
#pragma unroll
            for (int k = 0; k < 3; ++k)
              acc[i * 3 + k] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[i], bv[k], acc[i * 3 + k], 0, 0, 0);
        }
      }
      if (j == 0) {
        // Every load of this iteration is consumed here, before this cell's stores (a value still
        // in flight when they issue would be waited for behind them): the next cell's vertices and
        // bc bits go to LDS, its material values and the indices of the cell after it into registers
        if (ci + G < ncells) {
          if (tid < 24) s_xv[tid] = xval;
          put_bc(par ^ 1, bits);
        }
        cell_lame_from(F, la, lb, lam_n, mu_n);
        asm volatile("" ::"v"(gv2), "v"(nv2), "v"(lam_n), "v"(mu_n));
        gv1 = gv2;
        nv1 = nv2;
      }
      // D layout (f64 16x16x4): col = lane & 15, row = (lane >> 4) + 4 * r
      if constexpr (MODE == 2) {
        // block store for the row gather, Eb[c][a][b][3][3] with bc rows / columns zeroed: the
        // wave's 4 x 16 blocks of each r go through its own LDS staging and leave as contiguous
        // stores (512 B / 1 KB per instruction), instead of nine 72-B-strided stores per lane
        double* st = s_st[wave];
        const int nbv = min(16, NN - tb * 16);  // valid column blocks of this tile
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int a = ta * 16 + (lane >> 4) + 4 * r, b = tb * 16 + (lane & 15);
          if (a < NN && b < NN) {
            const double tr = acc[0][r] + acc[4][r] + acc[8][r];
            const uint32_t ra = s_bcn[par][a], rb = s_bcn[par][b];
            const uint32_t rm = (ra & 1u) | ((ra >> 7) & 2u) | ((ra >> 14) & 4u);
            const uint32_t cm = (rb & 1u) | ((rb >> 7) & 2u) | ((rb >> 14) & 4u);
#pragma unroll
            for (int i = 0; i < 3; ++i)
#pragma unroll
              for (int k = 0; k < 3; ++k) {
                const double v = lam * acc[i * 3 + k][r] + mu * acc[k * 3 + i][r] + (i == k ? mu * tr : 0.0);
                st[lane * 9 + i * 3 + k] = (((rm >> i) | (cm >> k)) & 1u) ? 0.0 : v;
              }
          }
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
          __builtin_amdgcn_wave_barrier();
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
          // row j of the 4: blocks [tb*16, tb*16 + nbv) of row a_j are contiguous in Eb
          if constexpr (NN % 16 == 0) {
            // whole 16-block rows (Q3): 4 x 72 16-B pairs, lane pair P = lane + 64 u of row P / 72,
            // stored with buffer stores whose offsets are per-lane constants (round 5: the generic
            // loop below spent ~60 VALU per 8-B store on its index arithmetic, and its store phase
            // took ~35 % of the cell's clocks)
            typedef int v4i __attribute__((ext_vector_type(4)));
            const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
                Ae + ((ci * NN + ta * 16 + 4 * r) * NN + tb * 16) * 9, 0, (3 * NN * 9 + 144) * 8, 0x00020000);
            const fa_dv2* s2 = reinterpret_cast<const fa_dv2*>(st);
            fa_dv2 v[5];
#pragma unroll
            for (int u = 0; u < 5; ++u) v[u] = s2[u < 4 || lane < 32 ? lane + 64 * u : 0];  // all reads first
#pragma unroll
            for (int u = 0; u < 5; ++u) {
              const int P = lane + 64 * u;
              if (u < 4 || P < 288) {
                const int j = P / 72, q = P - 72 * j;
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4i, v[u]), rs, (j * NN * 9 + 2 * q) * 8, 0, 0);
                store_guard1(v[u]);
              }
            }
          } else {
            const int nrow = nbv * 9;
            for (int t = lane; t < 4 * nrow; t += 64) {
              const int j = t / nrow, off = t - j * nrow;
              const int aj = ta * 16 + j + 4 * r;
              if (aj < NN) Ae[((ci * NN + aj) * NN + tb * 16) * 9 + off] = st[j * 144 + off];
            }
          }
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
          __builtin_amdgcn_wave_barrier();
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
        continue;
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int a = ta * 16 + (lane >> 4) + 4 * r, b = tb * 16 + (lane & 15);
        if (a >= NN || b >= NN) continue;
        double K[3][3];
        const double tr = acc[0][r] + acc[4][r] + acc[8][r];
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
          for (int k = 0; k < 3; ++k) K[i][k] = lam * acc[i * 3 + k][r] + mu * acc[k * 3 + i][r] + (i == k ? mu * tr : 0.0);
        if (MODE == 0) {
          double* out = Ae + ci * (int64_t)(3 * NN) * (3 * NN);
#pragma unroll
          for (int i = 0; i < 3; ++i)
#pragma unroll
            for (int k = 0; k < 3; ++k) out[(a * 3 + i) * (3 * NN) + b * 3 + k] = K[i][k];
          store_fence(K);
        } else if (MODE == 2) {  // block store for the row gather: Eb[c][a][b][3][3], bc rows/cols zeroed
          double* out = Ae + ((ci * NN + a) * NN + b) * 9;
          const int64_t na = cn[a], nb = cn[b];
#pragma unroll
          for (int i = 0; i < 3; ++i) {
            const bool ri = bc && bc[na * 3 + i];
#pragma unroll
            for (int k = 0; k < 3; ++k) out[i * 3 + k] = (ri || (bc && bc[nb * 3 + k])) ? 0.0 : K[i][k];
          }
        } else {
          const int64_t na = cn[a], nb = cn[b];
          if (na < A.row_begin || na >= A.row_end) continue;
          const int64_t sl = find_slot(A.indptr, A.indices, na, (int32_t)nb);
          if (sl < 0) {
            atomicOr(err, 1);
            continue;
          }
          double* dst = A.data + (sl - A.indptr[A.row_begin]) * 9;
#pragma unroll
          for (int i = 0; i < 3; ++i) {
            if (bc && bc[na * 3 + i]) continue;
#pragma unroll
            for (int k = 0; k < 3; ++k) {
              if (bc && bc[nb * 3 + k]) continue;
              unsafeAtomicAdd(dst + i * 3 + k, K[i][k]);
            }
          }
        }
      }
    }
    lam = lam_n;
    mu = mu_n;
  }
}

static int launch_hex_mfma(int mode, const fa_mesh* mesh, const MeshView& M, const FormView& F, const DevTables& T,
                           int64_t c0, int64_t nc, double* Ae, const BsrView& A, const int8_t* bc, int* derr,
                           hipStream_t s, bool* handled) {
  *handled = false;
  if (mesh->cell_type != FA_HEXAHEDRON || F.kind != FA_LINEAR_ELASTICITY || nc <= 0) return FA_OK;
  *handled = true;
  const int grid = (int)std::min<int64_t>(nc, kMaxBlocks);
#define HEXL(NN, NQ)                                                                                          \
  do {                                                                                                        \
    constexpr int thr = hex_threads(NN);                                                                      \
    if (mode == 0) k_hex_mfma<NN, NQ, 0><<<grid, thr, 0, s>>>(M, F, T, c0, nc, Ae, A, bc, derr);               \
    else if (mode == 2) k_hex_mfma<NN, NQ, 2><<<grid, hex_threads_m(NN, 2), 0, s>>>(M, F, T, c0, nc, Ae, A, bc, derr); \
    else k_hex_mfma<NN, NQ, 1><<<grid, thr, 0, s>>>(M, F, T, c0, nc, Ae, A, bc, derr);                        \
  } while (0)
  // the default (UFL-estimated) rules: Q1 2^3, Q2 3^3, Q3 4^3 points
  if (mesh->nn == 8 && T.nq == 8) HEXL(8, 8);
  else if (mesh->nn == 27 && T.nq == 27) HEXL(27, 27);
  else if (mesh->nn == 64 && T.nq == 64) HEXL(64, 64);
  else {
    *handled = false;
    return FA_OK;
  }
#undef HEXL
  LAUNCH_CHECK();
  return FA_OK;
}

// set bc diagonal entries (after the gather / scatter)
template <int GD, int WPT>
__global__ __launch_bounds__(256) void k_bc_diag(BsrView A, int64_t nnodes, const int8_t* __restrict__ bc, double diag,
                                                int* err) {
  // dolfinx set_diagonal over the window's rows. A workgroup scans 64 KB of markers (16 aligned 16-B
  // words per thread, all loads in flight at once), queues the constrained dofs in LDS and then
  // resolves them (find_slot: ~7 dependent loads) on all its lanes at once. Round 5: a thread per dof
  // left about one active lane per wave, and config E's ~1 M constrained dofs of 202 M took 0.41 ms
  // (now 0.26).
  constexpr int NT = 256, QCAP = 4096;
  constexpr int64_t SPAN = 16 * NT * WPT;
  __shared__ int64_t q[QCAP];
  __shared__ int qn;
  const int64_t d0 = A.row_begin * GD, d1 = A.row_end * GD;
  const int64_t a0 = (int64_t)(((uintptr_t)bc + (uintptr_t)d0) & ~(uintptr_t)15) - (int64_t)(uintptr_t)bc;
  // (one search per node instead of per dof, the node queued by its first constrained dof, measured
  // 0.32 vs 0.26 ms on config E: the first-dof test's byte loads in the scan cost more than it saved;
  // round 6: the marker bytes taken from the loaded words instead of loaded again, 0.30 vs 0.26 ms)
  auto resolve = [&](int64_t n) {
    const int64_t r = n / GD;
    const int i = (int)(n % GD);
    const int64_t s = find_slot(A.indptr, A.indices, r, (int32_t)r);
    if (s < 0) atomicOr(err, 2);
    else A.data[(s - A.indptr[A.row_begin]) * GD * GD + i * GD + i] = diag;
  };
  for (int64_t base = a0 + (int64_t)blockIdx.x * SPAN; base < d1; base += (int64_t)gridDim.x * SPAN) {
    if (threadIdx.x == 0) qn = 0;
    __syncthreads();
    uint4 w[WPT];
#pragma unroll
    for (int it = 0; it < WPT; ++it) {  // whole words inside the window (and the array) are loaded
      const int64_t o = base + 16 * (it * NT + (int64_t)threadIdx.x);
      w[it] = (o >= d0 && o + 16 <= d1) ? *reinterpret_cast<const uint4*>(bc + o) : make_uint4(1u, 1u, 1u, 1u);
    }
#pragma unroll
    for (int it = 0; it < WPT; ++it) {
      if ((w[it].x | w[it].y | w[it].z | w[it].w) == 0u) continue;
      const int64_t o = base + 16 * (it * NT + (int64_t)threadIdx.x);
      for (int k = 0; k < 16; ++k) {
        const int64_t n = o + k;
        if (n < d0 || n >= d1 || !bc[n]) continue;
        const int slot = atomicAdd(&qn, 1);
        if (slot < QCAP) q[slot] = n;
        else resolve(n);  // a pass with more constrained dofs than the queue holds
      }
    }
    __syncthreads();
    const int cnt = min(qn, QCAP);
    for (int t = threadIdx.x; t < cnt; t += NT) resolve(q[t]);
    __syncthreads();  // the queue is read before the next pass resets it
  }
}
// k_bc_diag over a window of n dofs: 64 KB of markers per workgroup pass, or 4 KB when that leaves
// fewer than ~2,000 workgroups (config C's 5 M dofs: 80 workgroups of 64 KB resolved ~1,000 dofs each,
// 0.068 ms; a thread per dof had taken 0.021 ms)
template <int GD>
static void launch_bc_diag(const BsrView& A, int64_t n, const int8_t* bc, double diag, int* err, hipStream_t s) {
  auto grid = [](int64_t n, int64_t span) {
    return (int)std::max<int64_t>(1, std::min<int64_t>((n + 16 + span - 1) / span + 1, (1 << 24) - 8));
  };
  if (n >= 2048ll * 65536) k_bc_diag<GD, 16><<<grid(n, 65536), 256, 0, s>>>(A, 0, bc, diag, err);
  else k_bc_diag<GD, 1><<<grid(n, 4096), 256, 0, s>>>(A, 0, bc, diag, err);
}

// ------------------------------------------------------------------------------------ gather kernel
// Two launches per assembly:
//  1. k_cell_records: one thread per cell packs what every (row, cell) item of the gather
//     needs into a small record — inverse Jacobian(s), |det J|, lambda, mu (or, for the damage
//     law, physical gradients, weight and the tangent "hook") — plus a 32-bit mask of the
//     cell's constrained dofs (bit b*GD+j). A streaming pass: reads the cell's geometry once.
//  2. k_gather: one workgroup per row chunk (XCD-aware order: chunks of one XCD are
//     contiguous so its L2 holds the cells they share). Items (adjacency entry, column group)
//     read one record + the column node ids, build 3x3 blocks in registers and add them into
//     the LDS copy of the chunk; the chunk is then stored with coalesced plain stores.
constexpr int FA_GATHER_LDS = 32768;  // 4 workgroups / CU with k_gather_lin's table (E: 44.3 vs 45.3 ms at 28672)
static constexpr int kGatherLdsValues = FA_GATHER_LDS;  // accumulator bytes per workgroup (4 WG / CU)
// neo-Hookean gather (2 workgroups / CU, VGPR-bound): a larger accumulator, and chunks capped at
// 256 / NSPLIT adjacency entries so one chunk's items fill the workgroup's 256 lanes once
// (fa_plan_gather_form); with the default plan ~96 entries -> 192 items left a wave idle
constexpr int FA_GATHER_LDS_NEO = 46080;
static constexpr int kGatherLdsNeo = FA_GATHER_LDS_NEO;
constexpr int FA_NEO_NSPLIT = 2;  // neo-Hookean column items of 5 columns (E-neo at 2 waves / SIMD, round 2: NSPLIT 2
                                  // 342 ms, 5 at 3 waves 349, 10 at 4 waves 461; round 5: whole entries, 256
                                  // per chunk in a 72 KB accumulator, 64.1 vs 64.2 ms, plan 2.5 vs 1.5 s)
// the neo-Hookean gather's item split per element (launch_gather's instantiations; its plans are
// ordered for it and capped at 256 / split entries per chunk)
static int neo_nsplit(int ct, int p) {
  return ct == FA_TETRAHEDRON && p == 2 ? FA_NEO_NSPLIT : (ct == FA_TRIANGLE && p == 2 ? 2 : 1);
}
constexpr int FA_GATHER_ENTRY_CAP = 512;  // adjacency entries per chunk of the default plan (512 = the LDS arrays' cap)
// blocks of the accumulator of a gather kernel (the plan's chunks must fit it)
__host__ __device__ constexpr int gather_maxb(bool neo, int bs2) {
  return (neo ? kGatherLdsNeo : kGatherLdsValues) / (8 * bs2) < 1023 ? (neo ? kGatherLdsNeo : kGatherLdsValues) / (8 * bs2)
                                                                      : 1023;
}
// k_gather_lin for P1 simplices: chunks are entry-bound (config C: ~160 blocks), so a 16 KB
// accumulator and more resident waves
constexpr int kLinLdsP1 = 16384;
constexpr int kLinWavesP1 = 4;
__host__ __device__ constexpr int lin_maxb(int gd, int nn) {
  return nn == gd + 1 ? kLinLdsP1 / (8 * gd * gd) : gather_maxb(false, gd * gd);
}
static constexpr int kGatherMaxAdj = 512;       // adjacency entries per chunk
static constexpr int kGatherMaxRows = 128;      // rows per chunk

// gather variant whose blocks come from a per-cell block store [cell][a][b][GD][GD] (hexahedra:
// written by the MFMA kernel) instead of being computed from a record
constexpr int MAT_BLOCKS = 9;
// MAT_BLOCKS: adjacency entries in flight per wave (one wave per entry, coalesced block-store reads):
// measured 1 / 2 / 3 -> Dmfma 50.0 / 46.0 / 47.3 ms
constexpr int kEbUnroll = 2;
// linear elasticity with one Poisson ratio for all cells (E per cell): lam / mu = r is uniform, so
// lam G + mu G^T = mu |J| Ji^T (r Ahat + Ahat^T) Ji; the record holds s Ji with s^2 = mu |J|
// (and the sign of mu |J|), the table B_ab = r Ahat_ab + Ahat_ab^T, and
// K = H + tr(H) / (1 + r) I with H = (s Ji)^T B (s Ji): 19 fewer FP64 ops per block
constexpr int MAT_LINU = 10;
// linear elasticity, uniform nu, on affine tensor cells (parallelograms / parallelepipeds): the
// uniform-nu record of an affine simplex (s Ji, sign) and a reference tensor that factorises into
// 1-D matrices (tensor_1d_mats), computed per block instead of read from a table -- the simplex
// gather for Q1-Q3 hexahedra of a structured mesh, with no element-matrix store
constexpr int MAT_AFFT = 11;

template <int GD, int NV, int NQ, int MAT>
struct Rec {
  static constexpr bool SIMP = (NV == GD + 1) || MAT == MAT_AFFT;  // affine: one Jacobian per cell
  // LIN simplex: Ji[GD*GD], wdet, lam, mu | LINU (simplex): s Ji[GD*GD], sign(mu wdet) |
  // LIN tensor: NQ x (Ji[GD*GD], wdet), lam, mu | DAMAGE (P1 tri): g[3][2], w, H[3][3]
  static constexpr int RAW = MAT == MAT_BLOCKS ? 2
                             : (MAT == MAT_LINU || MAT == MAT_AFFT) ? GD * GD + 1
                             : MAT == FA_ASYM_DAMAGE ? 16
                                                     : (SIMP ? GD * GD + 3 : NQ * (GD * GD + 1) + 2);
  static constexpr int SIZE = (RAW + 1) & ~1;  // even: 16-byte aligned records
  __host__ __device__ static constexpr int64_t head(int64_t c) { return c * SIZE; }
  __host__ __device__ static constexpr int64_t count(int64_t nc) { return nc * SIZE; }
};

struct GatherArgs {
  MeshView M;
  FormView F;
  BsrView A;
  const int64_t* adj_ptr;
  const int32_t* adj_idx;
  const int64_t* row_start;
  const int32_t* corder;   // [nchunks] visiting order (fa_plan_locality) or NULL (row order)
  const int64_t* chunk_b;  // [nchunks + 1] indptr[row_start[c]] (k_chunk_desc)
  const int64_t* chunk_a;  // [nchunks + 1] adj_ptr[row_start[c]]
  const int64_t* chunk_desc;  // the plan's cached k_gather_lin chunk arrays (fa_plan_chunk_desc), or NULL
  int64_t nchunks;
  int32_t plan_maxb;        // largest block count of a chunk of the plan (checked against the kernel's)
  int32_t plan_maxadj;      // largest adjacency count of a chunk of the plan
  unsigned long long* ctr;  // [8] per-XCD chunk counters (dynamic persistent grid), or NULL
  const uint16_t* slots;  // optional [adjacency entry][NN] position of the block within its row
  int slot_order;         // 0, or the NSPLIT whose item order fa_plan_order baked into `slots`
  // positional plan (fa_plan_order with an entry buffer): each chunk's adjacency entries in the
  // plan's bank-balanced order; `slots` is then indexed by that position and holds chunk-relative
  // block positions, so items need neither the entry permutation nor their row
  const int32_t* eadj;
  const int8_t* bc;
  double diag;
  const double* tab;  // device tables: wq | dphi | gdphi
  const double* ahat; // simplex reference tensor [nn][nn][GD][GD] (MAT_LINU: the table B)
  double trc;         // MAT_LINU: 1 / (1 + lam / mu)
  double rlm;         // MAT_LINU: lam / mu
  int affine;         // every cell affine (plan cell_flags & FA_PLAN_AFFINE): tensor cells may use MAT_AFFT
  const double* t1d;  // MAT_AFFT: 1-D matrices S, M, C [3][p+1][p+1]
  const double* lat;  // MAT_AFFT: node lattice codes a0 + 8 a1 + 64 a2
  const double* rec;  // [ncells][Rec::SIZE]
  const uint32_t* bcmask;  // [ncells] or NULL
  const double* xpack;      // fused P1 records (k_gather_lin FUSE): [nnodes][4] = the node's coordinates
                            // and its constrained-dof bits (as the bits of a double), k_pack_nodes
  int* err;
  // deterministic assembly (FA_DETERMINISTIC): k_gather_lin accumulates 64-bit fixed point (integer
  // LDS atomics, order-independent sums); fixc bounds an item's block entries by fixc * rho^2,
  // rho = sum |record entries|
  int fix;
  double fixc;
  double amax;  // max |ahat| entry of the element (DevTables::amax)
  const uint64_t* pk;  // packed integer reference tensor (DevTables::pk) or NULL
  double pks, pkmax;   // its 1 / sqrt(D) and max |N|
  // contribution plan (fa_plan_contrib, k_gather_own) or NULL
  const int64_t* cw;       // [nchunks + 1] offsets of the chunks' word sections (u16 units)
  const int32_t* ccells;   // [nchunks][FA_OWN_CCAP] the chunk's distinct cells (-1 padded)
  const uint16_t* cwords;  // per chunk: 256 lane starts, then K x 256 contribution words
};

// The record of cell c for the gather (all kinds but the neo-Hookean tangents): see Rec.
template <int GD, int NN, int NV, int NQ, int MAT>
__device__ __forceinline__ void cell_record(const MeshView& M, const FormView& F, const double* __restrict__ tab, int64_t c,
                                            double (&r)[Rec<GD, NV, NQ, MAT>::SIZE]) {
  using R = Rec<GD, NV, NQ, MAT>;
#pragma unroll
  for (int k = 0; k < R::SIZE; ++k) r[k] = 0.0;
  if constexpr (MAT == FA_ASYM_DAMAGE) {
    double g[3][2], w, H[3][3];
    damage_cell(M, F, c, g, w, H);
#pragma unroll
    for (int a = 0; a < 3; ++a) { r[2 * a] = g[a][0]; r[2 * a + 1] = g[a][1]; }
    r[6] = w;
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j) r[7 + 3 * i + j] = H[i][j];
  } else if constexpr (MAT == MAT_LINU || MAT == MAT_AFFT) {
    static_assert(R::SIMP, "uniform-nu records: affine cells");
    double lam, mu;
    cell_lame(F, c, lam, mu);
    double Ji[GD][GD];
    const double s2 = mu * fabs(MAT == MAT_AFFT ? affine_tensor_geometry<GD, NV>(M, c, Ji) : simplex_geometry<GD>(M, c, Ji));
    const double sc = sqrt(fabs(s2));
#pragma unroll
    for (int i = 0; i < GD; ++i)
#pragma unroll
      for (int k = 0; k < GD; ++k) r[i * GD + k] = sc * Ji[i][k];
    r[GD * GD] = s2 < 0.0 ? -1.0 : 1.0;
  } else {
    double lam, mu;
    cell_lame(F, c, lam, mu);
    if constexpr (R::SIMP) {
      double Ji[GD][GD];
      double det = simplex_geometry<GD>(M, c, Ji);
#pragma unroll
      for (int i = 0; i < GD; ++i)
#pragma unroll
        for (int k = 0; k < GD; ++k) r[i * GD + k] = Ji[i][k];
      r[GD * GD] = fabs(det);
      r[GD * GD + 1] = lam;
      r[GD * GD + 2] = mu;
    } else {
      double xv[NV][GD];
      const int32_t* gv = M.geom + c * NV;
#pragma unroll
      for (int v = 0; v < NV; ++v)
#pragma unroll
        for (int i = 0; i < GD; ++i) xv[v][i] = M.x[(int64_t)gv[v] * GD + i];
      const double* gdphi = tab + NQ + NQ * NN * GD;
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        double Ji[GD][GD];
        double det = tensor_geometry<GD, NV>(xv, gdphi + q * NV * GD, Ji);
#pragma unroll
        for (int i = 0; i < GD; ++i)
#pragma unroll
          for (int k = 0; k < GD; ++k) r[q * (GD * GD + 1) + i * GD + k] = Ji[i][k];
        r[q * (GD * GD + 1) + GD * GD] = fabs(det);
      }
      r[NQ * (GD * GD + 1)] = lam;
      r[NQ * (GD * GD + 1) + 1] = mu;
    }
  }
}

// constrained-dof bits of cell c (bit b*GD+j), or "touches a constrained dof" for cells with more
// dofs than mask bits (the gather looks those up)
template <int GD, int NN>
__device__ __forceinline__ uint32_t cell_bcmask(const MeshView& M, const int8_t* __restrict__ bc, int64_t c) {
  uint32_t m = 0;
  const int32_t* cn = M.cells + c * NN;
  if constexpr (NN * GD <= 32) {
#pragma unroll
    for (int b = 0; b < NN; ++b) {
      int64_t n = cn[b];
#pragma unroll
      for (int j = 0; j < GD; ++j) m |= (bc[n * GD + j] ? 1u : 0u) << (b * GD + j);
    }
  } else {
    for (int b = 0; b < NN; ++b) {
      int64_t n = cn[b];
#pragma unroll
      for (int j = 0; j < GD; ++j) m |= bc[n * GD + j] ? 1u : 0u;
    }
  }
  return m;
}

// The uniform-nu record's last word is +-1 (the sign of mu |J|) with, for cells of <= 32 dofs, the
// cell's constrained-dof bits in its low 32 mantissa bits (k_cell_records_staged): its sign and its
// mask, without a separate mask load per item.
__device__ __forceinline__ double rec_sign(double w) { return copysign(1.0, w); }
__device__ __forceinline__ uint32_t rec_mask(double w) { return (uint32_t)__double_as_longlong(w); }

template <int GD, int NN, int NV, int NQ, int MAT>
__global__ __launch_bounds__(256) void k_cell_records(MeshView M, FormView F, const double* __restrict__ tab,
                                                      const int8_t* __restrict__ bc, double* __restrict__ rec,
                                                      uint32_t* __restrict__ bcmask) {
  using R = Rec<GD, NV, NQ, MAT>;
  for (int64_t c = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; c < M.ncells; c += (int64_t)gridDim.x * blockDim.x) {
  {
  double r[R::SIZE];
  cell_record<GD, NN, NV, NQ, MAT>(M, F, tab, c, r);
  double2* out = reinterpret_cast<double2*>(rec + c * R::SIZE);
#pragma unroll
  for (int k = 0; k < R::SIZE / 2; ++k) out[k] = make_double2(r[2 * k], r[2 * k + 1]);
  store_fence(r);
  }
  if (bcmask) bcmask[c] = cell_bcmask<GD, NN>(M, bc, c);
  }
}

// Records of at most 16 doubles (uniform-nu and general linear simplices, affine tensor cells, the
// damage law): a wave's 64 consecutive cells' records are one contiguous run; the lanes write them
// into wave-private LDS and the wave stores the run with 16 B per lane (a lane storing its own
// 80-B record touches one cache line per lane per store instruction). Config E: see DESIGN.md.
template <int GD, int NN, int NV, int NQ, int MAT>
__global__ __launch_bounds__(256) void k_cell_records_staged(MeshView M, FormView F, const double* __restrict__ tab,
                                                             const int8_t* __restrict__ bc, double* __restrict__ rec,
                                                             uint32_t* __restrict__ bcmask) {
  using R = Rec<GD, NV, NQ, MAT>;
  static_assert(R::SIZE <= 16, "staged records: small records");
  __shared__ __attribute__((aligned(16))) double sbuf[4][64 * R::SIZE];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  double* sb = sbuf[wave];
  for (int64_t cb = (int64_t)blockIdx.x * 256 + wave * 64; cb < M.ncells; cb += (int64_t)gridDim.x * 256) {
    const int64_t c = cb + lane;
    const bool valid = c < M.ncells;
    const int64_t cc = valid ? c : M.ncells - 1;
    double r[R::SIZE];
    cell_record<GD, NN, NV, NQ, MAT>(M, F, tab, cc, r);
    uint32_t m = 0u;
    if (bcmask && bc && valid) m = cell_bcmask<GD, NN>(M, bc, c);  // (bc NULL: k_rec_bcbits adds the bits)
    // the mask also rides in the sign word (rec_sign; affine tensor cells too: k_gather_lin reads them)
    if constexpr ((MAT == MAT_LINU || MAT == MAT_AFFT) && NN * GD <= 32)
      r[GD * GD] = __longlong_as_double(__double_as_longlong(r[GD * GD]) | (long long)m);
#pragma unroll
    for (int k = 0; k < R::SIZE; ++k) sb[lane * R::SIZE + k] = r[k];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int nv = (int)min<int64_t>(64, M.ncells - cb) * R::SIZE;  // even
    const double2* s2 = reinterpret_cast<const double2*>(sb);
    double2* d2 = reinterpret_cast<double2*>(rec + cb * R::SIZE);
    for (int t = lane; t < nv / 2; t += 64) {
      const fa_dv2 w = reinterpret_cast<const fa_dv2*>(s2)[t];
      reinterpret_cast<fa_dv2*>(d2)[t] = w;
      store_guard1(w);  // the next pass's LDS read returns into these registers
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (bcmask && valid) bcmask[c] = m;
  }
}

// The constrained-dof bits of the uniform-nu records from the constrained nodes' side (round 6): the
// records kernel then reads no dofmap (40 B per P2 tet of its ~98) and this kernel ORs each constrained
// node's bits into the records (and the mask array) of the cells around it through the node -> cell
// adjacency. A wave reads the markers of 8 x 64 consecutive nodes (lane = node, the 8 loads in flight
// together), then takes its constrained nodes one after the other with a lane per adjacency entry, so an
// atomic's latency is paid once per constrained node, not once per (node, cell) pair (a thread walking its
// node's ~24 cells alone: 0.37 ms on config E; per 16 marker bytes and component: 0.66 ms; a wave per 64
// nodes: 0.26 ms, one load latency per wave). The same bits as cell_bcmask: bit b * GD + j of cell c for
// its local node b, component j.
template <int GD, int NN, int RS>
__global__ __launch_bounds__(256) void k_rec_bcbits(const int64_t* __restrict__ adj_ptr, const int32_t* __restrict__ adj_idx,
                                                    const int8_t* __restrict__ bc, int64_t nnodes, double* __restrict__ rec,
                                                    uint32_t* __restrict__ bcmask) {
  static_assert(NN * GD <= 32, "bc bits of the record word");
  constexpr int U = 8;  // 64-node groups per wave pass: their marker loads in flight together
  const int lane = threadIdx.x & 63;
  const int64_t wid = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int64_t nwv = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t base = wid * (64 * U); base < nnodes; base += nwv * (64 * U)) {
    uint32_t nb[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t n = base + 64 * u + lane;
      nb[u] = 0u;
      if (n < nnodes) {
#pragma unroll
        for (int j = 0; j < GD; ++j) nb[u] |= (bc[n * GD + j] ? 1u : 0u) << j;
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      unsigned long long act = __ballot(nb[u] != 0u);
      while (act) {  // wave-uniform
        const int l = __ffsll(act) - 1;
        act &= act - 1;
        const uint32_t nbl = (uint32_t)__shfl((int)nb[u], l);
        const int64_t nn = base + 64 * u + l;
        const int64_t e0 = adj_ptr[nn], e1 = adj_ptr[nn + 1];
        for (int64_t e = e0 + lane; e < e1; e += 64) {
          const int64_t p = adj_idx[e];
          const int64_t c = p / NN;
          const uint32_t bits = nbl << ((int)(p % NN) * GD);
          atomicOr(reinterpret_cast<unsigned long long*>(rec + c * RS + GD * GD), (unsigned long long)bits);
          if (bcmask) atomicOr(bcmask + c, bits);
        }
      }
    }
  }
}

// 16 zero bytes to LDS, the zero made at the store (volatile): hoisted out of the gather's chunk
// loop, the compiler had kept the zero vector in scratch, and each reload waited vmcnt(0) -- for
// every chunk store still in flight (stores count in vmcnt)
__device__ __forceinline__ void lds_zero16(double* p) {
  uint32_t a, b, c, d;
  asm volatile("v_mov_b32 %0, 0\n\tv_mov_b32 %1, 0\n\tv_mov_b32 %2, 0\n\tv_mov_b32 %3, 0"
               : "=v"(a), "=v"(b), "=v"(c), "=v"(d));
  typedef uint32_t u4 __attribute__((ext_vector_type(4)));
  *reinterpret_cast<u4*>(p) = u4{a, b, c, d};
}

// Workgroup-uniform load through the scalar cache: a constant-address-space pointer lets the
// compiler emit s_load (counted by lgkmcnt) instead of a vector load, whose vmcnt wait would also
// drain every earlier vector load AND store of the wave (CDNA counts stores in vmcnt).
template <typename T>
__device__ __forceinline__ T sload(const T* p, int64_t i) {
  return ((const __attribute__((address_space(4))) T*)p)[i];
}

// binary search of `col` in cols[lo, hi) (LDS)
__device__ __forceinline__ int lds_find(const int32_t* cols, int lo, int hi, int32_t col) {
  int l = lo, h = hi - 1;
  while (l <= h) {
    int mid = (l + h) >> 1;
    int32_t cm = cols[mid];
    if (cm == col) return mid;
    if (cm < col) l = mid + 1;
    else h = mid - 1;
  }
  return -1;
}

// Position of `col` in the sorted cols[lo, hi): fixed-trip lower bound (niter = ceil(log2) of the
// chunk's longest row, wave-uniform), so lanes of different rows do not diverge; -1 if absent.
__device__ __forceinline__ int lds_slot(const int32_t* cols, int lo, int hi, int32_t col, int niter) {
  int l = lo, n = hi - lo;
  for (int k = 0; k < niter; ++k) {
    const int h = n >> 1;
    const int32_t cv = cols[l + h];  // unconditional read (in the chunk's slots): no branch
    l = ((h > 0) & (cv <= col)) ? l + h : l;
    n -= h;
  }
  const int32_t cv = cols[l];
  return ((n > 0) & (cv == col)) ? l : -1;
}

// lds_slot for NB columns of ONE row at once: the searches share the interval length, so the
// NB probes of each halving step are independent LDS reads issued together (one latency per
// step instead of NB).
template <int NB>
__device__ __forceinline__ void lds_slots(const int32_t* cols, int lo, int hi, const int32_t (&col)[NB], int niter,
                                          int (&sl)[NB]) {
  int n = hi - lo;
#pragma unroll
  for (int b = 0; b < NB; ++b) sl[b] = lo;
  for (int k = 0; k < niter; ++k) {
    const int h = n >> 1;
    int32_t cv[NB];
#pragma unroll
    for (int b = 0; b < NB; ++b) cv[b] = cols[sl[b] + h];
#pragma unroll
    for (int b = 0; b < NB; ++b) sl[b] = ((h > 0) & (cv[b] <= col[b])) ? sl[b] + h : sl[b];
    n -= h;
  }
  int32_t cv[NB];
#pragma unroll
  for (int b = 0; b < NB; ++b) cv[b] = cols[sl[b]];
#pragma unroll
  for (int b = 0; b < NB; ++b) sl[b] = ((n > 0) & (cv[b] == col[b])) ? sl[b] : -1;
}

// Add a GD x GD block into LDS slot s. rowm/colm: the constrained-dof bits of the block's row
// and column node (zero for almost every block: then no per-entry test).
template <int GD>
__device__ __forceinline__ void lds_add_block(double* acc, int s, double (&K)[GD][GD], uint32_t rowm,
                                              uint32_t colm) {
  // Constrained entries are zeroed (only in waves that hold one: a wave-uniform branch), then all
  // GD^2 adds are issued unconditionally. An add of 0.0 into a constrained diagonal entry that
  // another lane sets to `diag` concurrently is harmless: LDS atomics are indivisible, and
  // diag + 0.0 == diag.
  if (__any((rowm | colm) != 0u)) {
#pragma unroll
    for (int i = 0; i < GD; ++i)
#pragma unroll
      for (int jj = 0; jj < GD; ++jj)
        if (((rowm >> i) | (colm >> jj)) & 1u) K[i][jj] = 0.0;
  }
#pragma unroll
  for (int i = 0; i < GD; ++i)
#pragma unroll
    for (int jj = 0; jj < GD; ++jj) atomicAdd(&acc[s * (GD * GD) + i * GD + jj], K[i][jj]);
}

// Items are (adjacency entry, column-node group). NSPLIT groups split the cell's NN column
// nodes so that a chunk exposes enough independent items to all 256 lanes.
// min waves per SIMD of k_gather: 4 -> <= 128 VGPRs (16 waves / CU); measured best
constexpr int kGatherWaves = 4;
// chunks per chunk-counter atomic of k_gather's dynamic schedule: measured 1 50.7, 2 48.2, 8 48.2 ms
// (E); C 1.95 / 1.95 / 2.02
constexpr int kGatherBatch = 2;
// 16-B values per thread per store batch of k_gather's chunk stream (LDS reads issued together)
constexpr int kGatherStoreBatch = 4;
// Item -> lane order of the gather: consecutive adjacency entries belong to the same row and add
// into the same LDS slots, so entry jj of a chunk with na entries goes to position
// (jj * stride) mod na, stride coprime to na; (x * stride) mod na in 32-bit with a float
// quotient estimate (x < 2^24: off by <= 1). Shared by k_gather and the plan's k_order_slots.
__device__ __forceinline__ int gather_perm_stride(int na) {
  int st = 97;
  while (na % st == 0 && st > 1) st -= 2;
  return st;
}
__device__ __forceinline__ int gather_perm(int jj, int na, int st, float inv) {
  const int x = jj * st;
  int j = x - na * (int)((float)x * inv);
  return j < 0 ? j + na : (j >= na ? j - na : j);
}

template <int GD, int NN, int NV, int NQ, int NSPLIT, int MAT>
__global__ __launch_bounds__(256, kGatherWaves) void k_gather(GatherArgs P) {
  using R = Rec<GD, NV, NQ, MAT>;
  constexpr int BS2 = GD * GD;
  constexpr int MAXB = gather_maxb(false, BS2);
  // ordered slots pack (b << 10) | chunk-relative position: positions must stay below 1024
  static_assert(MAXB < 1024, "FA_GATHER_LDS too large for the packed ordered-slot map");
  constexpr bool SIMP = R::SIMP;
  constexpr int NBG = (NN + NSPLIT - 1) / NSPLIT;  // column nodes per item
  __shared__ double acc[(MAXB + 1) * BS2];  // + one sink slot for (erroneous) missing columns
  __shared__ int32_t cols[MAXB];
  __shared__ int32_t rowoff[kGatherMaxRows + 1];
  __shared__ uint8_t s_rowbc[kGatherMaxRows];  // constrained-dof bits of each chunk row
  __shared__ uint8_t adjrow[kGatherMaxAdj];
  static_assert(MAT != FA_NEO_HOOKEAN, "neo-Hookean forms: k_gather_neo");
  constexpr bool TAB = (MAT != MAT_BLOCKS) && !SIMP;  // quadrature tables staged in LDS
  __shared__ double s_w[TAB ? NQ : 1];
  __shared__ double s_dphi[TAB ? NQ * NN * GD : 1];
  constexpr bool AFFT = MAT == MAT_AFFT;
  __shared__ double s_ahat[SIMP && !AFFT ? NN * NN * BS2 : 1];
  constexpr int P1D = AFFT ? (NN == 8 || NN == 4 ? 2 : (NN == 27 || NN == 9 ? 3 : 4)) : 1;  // 1-D nodes
  __shared__ double s_t1d[AFFT ? 3 * P1D * P1D : 1];
  __shared__ int s_lat[AFFT ? NN : 1];

  const int tid = threadIdx.x;
  const int64_t abase = sload(P.A.indptr, P.A.row_begin);  // block index of the window's first value
  constexpr int NPC = (MAXB + 255) / 256;           // column indices per thread (metadata slice)
  constexpr int NPA = (kGatherMaxAdj + 255) / 256;  // adjacency entries per thread
  static_assert(kGatherMaxRows < 256, "one row offset per thread");
  __shared__ int32_t s_adj[kGatherMaxAdj];

  // XCD-aware chunk order: blocks b and b+8 share an XCD (round-robin dispatch), so XCD
  // (b % 8) walks the contiguous chunk range [(b % 8) * per, (b % 8 + 1) * per). A workgroup's
  // valid chunks are a prefix of its sequence vb = blockIdx.x + k * gridDim.x.
  const int64_t per = (P.nchunks + 7) / 8;
  const int64_t vstep = gridDim.x;  // gridDim.x % 8 == 0: vb % 8 == blockIdx.x % 8
  auto chunk_of = [&](int64_t v) -> int64_t {
    if (v >= 8 * per) return P.nchunks;
    const int64_t c = (v % 8) * per + v / 8;
    return c < P.nchunks ? (P.corder ? (int64_t)P.corder[c] : c) : P.nchunks;
  };
  // Chunk sequence of this workgroup. Static (P.ctr == NULL): chunk_of(blockIdx.x + k*gridDim.x).
  // Dynamic (persistent grid): lane 0 takes the next chunk of its XCD's range from a per-XCD
  // counter (blockIdx.x % 8 = the XCD under round-robin dispatch; exhausted ranges are left for
  // the next one), three chunks ahead so the atomic's latency hides behind a chunk's work; the
  // index reaches the other lanes through LDS.
  __shared__ int64_t s_idx[3];
  // lane 0 takes FA_GATHER_BATCH consecutive chunks per counter atomic and serves them from this
  // batch [s_bat[0], s_bat[1]): the same-address atomics of an XCD's 128 workgroups on one L2
  // line were the kernel's throughput limit (one per ~80 ns per counter at one chunk per atomic)
  __shared__ int64_t s_bat[2];
  uint32_t qdone = 0u;  // lane 0: ranges found exhausted
  auto take_batch = [&](int q, unsigned long long c) {
    if ((int64_t)c < per) {
      const int64_t base = q * per + (int64_t)c;
      const int64_t end = min(q * per + min((int64_t)c + kGatherBatch, per), P.nchunks);
      if (base < end) {
        s_bat[0] = base;
        s_bat[1] = end;
        return;
      }
    }
    qdone |= 1u << q;
  };
  auto grab = [&]() -> int64_t {
#pragma unroll 1
    for (int t = 0; t < 9; ++t) {
      if (s_bat[0] < s_bat[1]) {
        const int64_t v = s_bat[0]++;
        return P.corder ? (int64_t)P.corder[v] : v;
      }
      if (t == 8) break;
      const int q = (int)((blockIdx.x + t) & 7);
      if ((qdone >> q) & 1u) continue;
      take_batch(q, atomicAdd(P.ctr + q, (unsigned long long)kGatherBatch));
    }
    return P.nchunks;
  };
  int64_t vb = blockIdx.x;
  int64_t idx0, idx1, idx2;
  if (P.ctr) {
    if (tid == 0) {
      s_bat[0] = s_bat[1] = 0;
      s_idx[0] = grab();
      s_idx[1] = grab();
      s_idx[2] = grab();
    }
    __syncthreads();
    idx0 = __builtin_amdgcn_readfirstlane((int)s_idx[0]);  // nchunks < 2^31 (checked on the host)
    idx1 = __builtin_amdgcn_readfirstlane((int)s_idx[1]);
    idx2 = __builtin_amdgcn_readfirstlane((int)s_idx[2]);
  } else {
    idx0 = chunk_of(vb);
    idx1 = chunk_of(vb + vstep);
    idx2 = chunk_of(vb + 2 * vstep);
  }
  if (idx0 >= P.nchunks) return;  // whole workgroup idle

  if constexpr (MAT == MAT_BLOCKS) {
  } else if constexpr (AFFT) {
    for (int t = tid; t < 3 * P1D * P1D; t += 256) s_t1d[t] = P.t1d[t];
    for (int t = tid; t < NN; t += 256) s_lat[t] = (int)P.lat[t];
  } else if constexpr (SIMP) {
    for (int t = tid; t < NN * NN * BS2; t += 256) s_ahat[t] = P.ahat[t];
  } else {
    for (int t = tid; t < NQ; t += 256) s_w[t] = P.tab[t];
    for (int t = tid; t < NQ * NN * GD; t += 256) s_dphi[t] = P.tab[NQ + t];
  }

  // Software pipeline over the workgroup's chunks: while chunk k is assembled, the metadata of
  // chunk k+1 (its column indices, row offsets, adjacency) is in flight into registers and the
  // descriptor of chunk k+2 is loaded, so a chunk starts with one exposed latency (its cells'
  // records) instead of four dependent ones (measured: the un-pipelined skeleton alone took
  // 46 of 84 ms on config E, tools/ablate.sh FA_ABL=6).
  // rows and adjacency entries fit 32 bits (the ABI checks ncells*nn < 2^31); block indices may not
  struct Desc { int64_t b0, b1; int32_t r0, r1, a0, a1; };
  auto load_desc = [&](int64_t c) -> Desc {
    return Desc{sload(P.chunk_b, c), sload(P.chunk_b, c + 1), (int32_t)sload(P.row_start, c),
                (int32_t)sload(P.row_start, c + 1), (int32_t)sload(P.chunk_a, c), (int32_t)sload(P.chunk_a, c + 1)};
  };
  int32_t pc[NPC], pj[NPA];
  // row / adjacency pointers: low 32 bits only (differences within a chunk are < 2^31)
  uint32_t prow = 0, pa0 = 0, pa1 = 0;
  uint32_t pbc[GD];  // raw constrained-dof bytes of row tid, combined in stage
  const uint32_t* indptr_lo = reinterpret_cast<const uint32_t*>(P.A.indptr);
  const uint32_t* adjptr_lo = reinterpret_cast<const uint32_t*>(P.adj_ptr);
  const int32_t* adj_src = P.eadj ? P.eadj : P.adj_idx;  // positional plan: entries in its order
  // Loads at clamped indices, unconditionally and with no use of their values here: a
  // per-load "load or constant" select makes hipcc branch around each load and wait for it,
  // which serialises the prefetch; stage() ignores the lanes past the chunk's counts.
  auto fetch = [&](const Desc& d) {
    const int nb_ = (int)(d.b1 - d.b0), nr_ = (int)(d.r1 - d.r0), na_ = (int)(d.a1 - d.a0);
    if (nb_ > 0) {
#pragma unroll
      for (int k = 0; k < NPC; ++k) pc[k] = P.A.indices[d.b0 + min(tid + 256 * k, nb_ - 1)];
    }
    const int rr = min(tid, nr_), rr1 = min(tid + 1, nr_);
    prow = indptr_lo[2 * (d.r0 + rr)];
    pa0 = adjptr_lo[2 * (d.r0 + rr)];
    pa1 = adjptr_lo[2 * (d.r0 + rr1)];
    if (P.bc && nr_ > 0) {
      const uint8_t* bp = reinterpret_cast<const uint8_t*>(P.bc) + (d.r0 + min(tid, nr_ - 1)) * GD;
#pragma unroll
      for (int i = 0; i < GD; ++i) pbc[i] = bp[i];
    } else {
#pragma unroll
      for (int i = 0; i < GD; ++i) pbc[i] = 0u;
    }
    if (na_ > 0) {
#pragma unroll
      for (int k = 0; k < NPA; ++k) pj[k] = adj_src[d.a0 + min(tid + 256 * k, na_ - 1)];
    }
  };
  // Metadata of a chunk: registers -> LDS. Runs right after the previous chunk's items barrier
  // and BEFORE its store, so the wait for the prefetched registers does not also wait for the
  // store's writes (vmcnt counts stores, and the store loop's trip count is not static).
  auto stage_meta = [&](const Desc& d) {
    const int nb_ = (int)(d.b1 - d.b0), nr_ = (int)(d.r1 - d.r0), na_ = (int)(d.a1 - d.a0);
    if (tid < nr_) {
      uint32_t bits = 0u;
#pragma unroll
      for (int i = 0; i < GD; ++i) bits |= (pbc[i] != 0u ? 1u : 0u) << i;
      s_rowbc[tid] = (uint8_t)bits;
    }
#pragma unroll
    for (int k = 0; k < NPC; ++k) {
      const int t = tid + 256 * k;
      if (t < nb_) cols[t] = pc[k];
    }
    if (tid <= nr_) rowoff[tid] = (int)(prow - (uint32_t)d.b0);
    if (tid < nr_) {
      const int j0 = (int)(pa0 - (uint32_t)d.a0), j1 = (int)(pa1 - (uint32_t)d.a0);
      for (int j = j0; j < j1; ++j) adjrow[j] = (uint8_t)tid;
    }
#pragma unroll
    for (int k = 0; k < NPA; ++k) {
      const int t = tid + 256 * k;
      if (t < na_) s_adj[t] = pj[k];
    }
  };
  auto zero_acc = [&](const Desc& d) {  // after the barrier that follows the previous store
    const int nb_ = (int)(d.b1 - d.b0);
    const int nv2 = (nb_ * BS2 + 1) >> 1;  // acc holds (MAXB + 1) blocks: the odd tail fits
    for (int t = tid; t < nv2; t += 256) lds_zero16(acc + 2 * t);
  };

  // consecutive adjacency entries belong to the same row and add into the same LDS slots (the
  // diagonal block of a vertex row gets ~24 adds); a stride coprime to na spreads rows over
  // lanes (measured +16 % on config E at n = 120). The NSPLIT parts of one entry stay on
  // neighbouring lanes (they read the same cell record).
  // kernels that can run a positional plan (the ordered-slot affine-simplex elasticity path)
  constexpr bool POSM = (MAT == 0 || MAT == MAT_LINU || (MAT == MAT_AFFT && NN * GD <= 32)) && SIMP && NN % NSPLIT == 0;
  auto perm_stride = [&](int na_) { return gather_perm_stride(na_); };
  auto perm = [&](int jj, int na_, int st, float inv) { return gather_perm(jj, na_, st, inv); };
  Desc cur = load_desc(idx0);
  fetch(cur);
  stage_meta(cur);
  zero_acc(cur);
  int64_t nchunk = idx1;   // chunk k+1 (its descriptor is loaded, its metadata staged next)
  int64_t nnchunk = idx2;  // chunk k+2 (its descriptor is loaded during chunk k)
  Desc nxt = nchunk < P.nchunks ? load_desc(nchunk) : cur;
  __syncthreads();
  int kpar = 0;
  for (;;) {
  // chunk k+3: lane 0 issues the counter atomic here and resolves it after the items, so the
  // wait for its return (a vmcnt wait) does not head the chunk
  unsigned long long gcand = 0ull;
  int gq = -1;
  if (P.ctr && tid == 0 && nnchunk < P.nchunks && s_bat[0] >= s_bat[1]) {  // batch used up
    for (int t = 0; t < 8; ++t) {
      const int q = (int)((blockIdx.x + t) & 7);
      if (!((qdone >> q) & 1u)) { gq = q; break; }
    }
    if (gq >= 0) gcand = atomicAdd(P.ctr + gq, (unsigned long long)kGatherBatch);
  }

  if (nchunk < P.nchunks) fetch(nxt);  // lands while this chunk is assembled
  Desc nn2;  // chunk k+2's descriptor: loaded after the items (scalar loads), used from the next chunk on

  const int64_t r0 = cur.r0;
  const int nrows = (int)(cur.r1 - cur.r0);
  const int64_t b0 = cur.b0;
  const int nb = (int)(cur.b1 - cur.b0);
  const int64_t a0 = cur.a0;
  const int na = (int)(cur.a1 - cur.a0);
  // fixed trip count of the in-kernel slot search: enough halvings for any row of a chunk
  // (<= MAXB blocks); extra ones are no-ops once the interval has one entry
  constexpr int niter = 32 - __builtin_clz((unsigned)MAXB);
  int bad = 0;
  // Dirichlet diagonals (dolfinx set_diagonal) before the items: no item adds into a constrained
  // dof's diagonal entry (its row bit masks the add), so this needs no barrier. The block-store
  // variant adds pre-zeroed entries unmasked and sets them after the items instead.
  if (MAT != MAT_BLOCKS && P.bc) {
    for (int t = tid; t < nrows * GD; t += 256) {
      const int lr = t / GD, i = t % GD;
      if (!((s_rowbc[lr] >> i) & 1u)) continue;
      const int s = lds_find(cols, rowoff[lr], rowoff[lr + 1], (int32_t)(r0 + lr));
      if (s < 0) { atomicOr(P.err, 2); continue; }
      acc[s * BS2 + i * GD + i] = P.diag;
    }
  }

  const int nitems = na * NSPLIT;
  const int stride = perm_stride(na);
  const float inv_n = 1.0f / (float)na;
  auto item = [&](const int it0) {
    const int part = it0 % NSPLIT;
    // positional plan: entries are staged in the plan's order and slots are chunk-relative
    const bool posm = POSM && P.eadj != nullptr;
    const int j = posm ? it0 / NSPLIT : perm(it0 / NSPLIT, na, stride, inv_n);
    const int32_t pflat = s_adj[j];
    const int64_t c = pflat / NN;
    const int aloc = pflat % NN;
    const int lr = posm ? 0 : adjrow[j];
    const int lo = posm ? 0 : rowoff[lr], hi = posm ? 0 : rowoff[lr + 1];
    // one record + the column nodes + the bc mask: all independent loads, issued together
    // registers: tensor cells read their per-q records in the q loop
    constexpr int RL = SIMP || MAT == FA_ASYM_DAMAGE ? R::SIZE : 2;
    double r[RL];
    int32_t cn[NBG];
    uint32_t mask;
    {
    if constexpr (MAT != MAT_BLOCKS) {
      const double2* rp = reinterpret_cast<const double2*>(P.rec + R::head(c));
#pragma unroll
      for (int k = 0; k < RL / 2; ++k) {
        double2 v = rp[k];
        r[2 * k] = v.x;
        r[2 * k + 1] = v.y;
      }
    }
    if (!P.slots) {  // column node ids: only the in-kernel slot search needs them
#pragma unroll
      for (int bb = 0; bb < NBG; ++bb) {
        const int b = part * NBG + bb;
        cn[bb] = b < NN ? P.M.cells[c * NN + b] : -1;
      }
    }
    mask = P.bcmask ? P.bcmask[c] : 0u;
    }

    if constexpr (MAT == MAT_BLOCKS) {
      const double* Eb = P.rec + ((int64_t)c * NN + aloc) * NN * BS2;  // bc already applied
#pragma unroll 1
      for (int bb = 0; bb < NBG; ++bb) {
        const int b = part * NBG + bb;
        if (b >= NN) break;
        int s = P.slots ? lo + (int)P.slots[(a0 + j) * NN + b] : lds_slot(cols, lo, hi, cn[bb], niter);
        bad |= s < 0;
        s = s < 0 ? MAXB : s;
#pragma unroll
        for (int e = 0; e < BS2; ++e) atomicAdd(&acc[s * BS2 + e], Eb[b * BS2 + e]);
      }
    } else if constexpr (MAT == FA_ASYM_DAMAGE) {
      double H[3][3];
#pragma unroll
      for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int k = 0; k < 3; ++k) H[i][k] = r[7 + 3 * i + k];
      const double w = r[6];
      double ga[2] = {r[2 * aloc], r[2 * aloc + 1]};
#pragma unroll
      for (int bb = 0; bb < NBG; ++bb) {
        const int b = part * NBG + bb;
        if (b >= NN) break;
        double gb[2] = {r[2 * b], r[2 * b + 1]};
        double K[2][2];
        damage_block(ga, gb, w, H, K);
        int s = P.slots ? lo + (int)P.slots[(a0 + j) * NN + b] : lds_slot(cols, lo, hi, cn[bb], niter);
        bad |= s < 0;
        s = s < 0 ? MAXB : s;
        lds_add_block<2>(acc, s, K, (mask >> (aloc * 2)) & 3u, (mask >> (b * 2)) & 3u);
      }
    } else if constexpr (SIMP) {
      // affine simplex: G_ab = |J| Ji^T Ahat_ab Ji  (reference-tensor form)
      constexpr bool LINU = MAT == MAT_LINU || MAT == MAT_AFFT;
      // LINU: r = s Ji, r[BS2] = sign; LIN: r = Ji, |J|, lam, mu
      const double wdet = LINU ? 1.0 : r[BS2], lam = LINU ? 0.0 : r[LINU ? 0 : BS2 + 1] * wdet,
                   mu = LINU ? 0.0 : r[LINU ? 0 : BS2 + 2] * wdet;
      const bool negw = LINU && __any(r[BS2] < 0.0);  // wave-uniform: a cell with mu |J| < 0
      int sl[NBG];  // slots of the item's column nodes, searched together
      // their local column indices b, 6 bits each (the plan's order when slot_order is set)
      static_assert(NBG * 6 <= 64 && NN <= 64, "packed column list");
      uint64_t bcp = 0;
#pragma unroll
      for (int bb = 0; bb < NBG; ++bb) bcp |= (uint64_t)(part * NBG + bb) << (6 * bb);
      if (P.slots && P.slot_order) {  // (b << 10) | position, in bank-conflict-aware order
#pragma unroll
        for (int bb = 0; bb < NBG; ++bb) {
          const int v = (int)P.slots[(a0 + j) * NN + part * NBG + bb];
          sl[bb] = lo + (v & 1023);
          bcp = (bcp & ~((uint64_t)63 << (6 * bb))) | ((uint64_t)(v >> 10) << (6 * bb));
        }
      } else if (P.slots) {
#pragma unroll
        for (int bb = 0; bb < NBG; ++bb)
          sl[bb] = part * NBG + bb < NN ? lo + (int)P.slots[(a0 + j) * NN + part * NBG + bb] : 0;
      } else {
        lds_slots<NBG>(cols, lo, hi, cn, niter, sl);
      }
      // constrained-dof bits: from the cell's mask, or -- cells with more dofs than mask bits -- from
      // the chunk row's bits and the column node's markers (only in waves holding such a cell)
      constexpr bool BIGM = NN * GD > 32;
      const uint32_t rowm = BIGM ? (mask ? (uint32_t)s_rowbc[lr] : 0u) : (mask >> (aloc * GD)) & ((1u << GD) - 1);
      const double* Ah0 = s_ahat + aloc * NN * BS2;
      const int alat = AFFT ? s_lat[aloc] : 0;
#pragma unroll 1
      for (int bb = 0; bb < NBG; ++bb) {
        if (NN % NSPLIT != 0 && part * NBG + bb >= NN) break;
        const int b = (int)(bcp & 63);  // rolled loop: shift the column list like the slot list
        bcp >>= 6;
        double Ahc[BS2];
        if constexpr (AFFT) {
          // reference tensor of an affine tensor cell from the 1-D matrices, then the uniform-nu
          // table entry B = (lam/mu) Ahat + Ahat^T
          const int blat = s_lat[b];
          double Sd[GD], Md[GD], Cd[GD], Ctd[GD];
#pragma unroll
          for (int d = 0; d < GD; ++d) {
            const int ad = (alat >> (3 * d)) & 7, bd = (blat >> (3 * d)) & 7;
            Sd[d] = s_t1d[ad * P1D + bd];
            Md[d] = s_t1d[P1D * P1D + ad * P1D + bd];
            Cd[d] = s_t1d[2 * P1D * P1D + ad * P1D + bd];
            Ctd[d] = s_t1d[2 * P1D * P1D + bd * P1D + ad];
          }
          double A[GD][GD];
#pragma unroll
          for (int jd = 0; jd < GD; ++jd)
#pragma unroll
            for (int ld = 0; ld < GD; ++ld) {
              double v = 1.0;
#pragma unroll
              for (int d = 0; d < GD; ++d)
                v *= (d == jd && d == ld) ? Sd[d] : (d == jd ? Cd[d] : (d == ld ? Ctd[d] : Md[d]));
              A[jd][ld] = v;
            }
#pragma unroll
          for (int i = 0; i < GD; ++i)
#pragma unroll
            for (int k = 0; k < GD; ++k) Ahc[i * GD + k] = fma(P.rlm, A[i][k], A[k][i]);
        } else {
#pragma unroll
          for (int e = 0; e < BS2; ++e) Ahc[e] = Ah0[b * BS2 + e];
        }
        const double* Ahp = Ahc;
        double T[GD][GD];  // T = Ahat Ji
#pragma unroll
        for (int i = 0; i < GD; ++i)
#pragma unroll
          for (int d = 0; d < GD; ++d) {
            double t = Ahp[i * GD] * r[d];
#pragma unroll
            for (int k = 1; k < GD; ++k) t = fma(Ahp[i * GD + k], r[k * GD + d], t);
            T[i][d] = t;
          }
        double G[GD][GD];  // G = Ji^T T
#pragma unroll
        for (int e = 0; e < GD; ++e)
#pragma unroll
          for (int d = 0; d < GD; ++d) {
            double g = r[e] * T[0][d];
#pragma unroll
            for (int i = 1; i < GD; ++i) g = fma(r[i * GD + e], T[i][d], g);
            G[e][d] = g;
          }
        double K[GD][GD];
        if constexpr (LINU) {
          double tr = G[0][0];
#pragma unroll
          for (int i = 1; i < GD; ++i) tr += G[i][i];
          tr *= P.trc;
#pragma unroll
          for (int i = 0; i < GD; ++i)
#pragma unroll
            for (int k = 0; k < GD; ++k) K[i][k] = i == k ? G[i][k] + tr : G[i][k];
          if (negw) {
            const double sg = rec_sign(r[BS2]);
#pragma unroll
            for (int i = 0; i < GD; ++i)
#pragma unroll
              for (int k = 0; k < GD; ++k) K[i][k] *= sg;
          }
        } else {
          lin_block<GD>(G, lam, mu, K);
        }
        int s = sl[0];  // rolled loop: shift the slot list instead of indexing it
#pragma unroll
        for (int k = 0; k + 1 < NBG; ++k) sl[k] = sl[k + 1];
        bad |= s < 0;
        s = s < 0 ? MAXB : s;
        uint32_t colm;
        if constexpr (BIGM) {
          colm = 0u;
          if (mask && s < MAXB) {
            const int64_t nb_ = cols[s];
#pragma unroll
            for (int jd = 0; jd < GD; ++jd) colm |= (P.bc[nb_ * GD + jd] ? 1u : 0u) << jd;
          }
        } else {
          colm = (mask >> (b * GD)) & ((1u << GD) - 1);
        }
        lds_add_block<GD>(acc, s, K, rowm, colm);
      }
    } else {
      // non-affine tensor cells: J^-1 per quadrature point, read from the record as the rolled
      // q loop needs it; only the per-column accumulators G stay live
      const double* rq = P.rec + c * R::SIZE;
      const double lam = rq[NQ * (BS2 + 1)];
      const double mu = rq[NQ * (BS2 + 1) + 1];
      double G[NBG][GD][GD];
#pragma unroll
      for (int bb = 0; bb < NBG; ++bb)
#pragma unroll
        for (int i = 0; i < GD; ++i)
#pragma unroll
          for (int k = 0; k < GD; ++k) G[bb][i][k] = 0.0;
#pragma unroll 1
      for (int q = 0; q < NQ; ++q) {
        const double* Jq = rq + q * (BS2 + 1);
        double Jl[BS2 + 1];
#pragma unroll
        for (int e = 0; e <= BS2; ++e) Jl[e] = Jq[e];
        const double wd = s_w[q] * Jl[BS2];
        double ga[GD];
#pragma unroll
        for (int d = 0; d < GD; ++d) {
          double sgd = 0.0;
#pragma unroll
          for (int k = 0; k < GD; ++k) sgd += s_dphi[(q * NN + aloc) * GD + k] * Jl[k * GD + d];
          ga[d] = wd * sgd;
        }
#pragma unroll
        for (int bb = 0; bb < NBG; ++bb) {
          const int b = part * NBG + bb;
          if (b >= NN) break;
          double gb[GD];
#pragma unroll
          for (int d = 0; d < GD; ++d) {
            double sgd = 0.0;
#pragma unroll
            for (int k = 0; k < GD; ++k) sgd += s_dphi[(q * NN + b) * GD + k] * Jl[k * GD + d];
            gb[d] = sgd;
          }
#pragma unroll
          for (int i = 0; i < GD; ++i)
#pragma unroll
            for (int k = 0; k < GD; ++k) G[bb][i][k] += ga[i] * gb[k];
        }
      }
#pragma unroll
      for (int bb = 0; bb < NBG; ++bb) {
        const int b = part * NBG + bb;
        if (b >= NN) break;
        double K[GD][GD];
        lin_block<GD>(G[bb], lam, mu, K);
        int s = P.slots ? lo + (int)P.slots[(a0 + j) * NN + b] : lds_slot(cols, lo, hi, cn[bb], niter);
        bad |= s < 0;
        s = s < 0 ? MAXB : s;
        lds_add_block<GD>(acc, s, K, (mask >> (aloc * GD)) & ((1u << GD) - 1), (mask >> (b * GD)) & ((1u << GD) - 1));
      }
    }
  };
  {
    int it0 = tid;
    if constexpr (MAT == MAT_BLOCKS) {
      if (P.slots) {
        // element blocks: one wave per adjacency entry, its NN blocks (NN * 9 contiguous values of
        // Eb[c][a][.]) streamed with coalesced 8-B-per-lane loads, one LDS add per value (a lane's
        // block b = idx / 9 and entry e = idx % 9), instead of one lane reading NSPLIT whole blocks
        const int lane = tid & 63, wv = tid >> 6;
        constexpr int NEV = NN * BS2, NR = (NEV + 63) / 64;
        // kEbUnroll entries per wave in flight (their loads issued together)
        for (int j0 = wv * kEbUnroll; j0 < na; j0 += 4 * kEbUnroll) {
          double v[kEbUnroll][NR];
          int sl[kEbUnroll][NR], lo[kEbUnroll];
#pragma unroll
          for (int w = 0; w < kEbUnroll; ++w) {
            const int j = min(j0 + w, na - 1);
            const int32_t pflat = s_adj[j];
            const int64_t c = pflat / NN;
            const int aloc = pflat % NN;
            lo[w] = rowoff[adjrow[j]];
            const double* Eb = P.rec + ((int64_t)c * NN + aloc) * NEV;
            const uint16_t* sr = P.slots + ((int64_t)a0 + j) * NN;
#pragma unroll
            for (int r = 0; r < NR; ++r) {
              const int idx = min(lane + 64 * r, NEV - 1);
              v[w][r] = __builtin_nontemporal_load(Eb + idx);
              sl[w][r] = (int)sr[idx / BS2];
            }
          }
#pragma unroll
          for (int w = 0; w < kEbUnroll; ++w) {
            if (j0 + w >= na) break;
#pragma unroll
            for (int r = 0; r < NR; ++r) {
              const int idx = lane + 64 * r;
              if (idx < NEV) {
                const int b = idx / BS2, e = idx - b * BS2;
                atomicAdd(&acc[(lo[w] + sl[w][r]) * BS2 + e], v[w][r]);
              }
            }
          }
        }
      } else {
        for (; it0 < nitems; it0 += 256) item(it0);
      }
    } else {
      for (; it0 < nitems; it0 += 256) item(it0);
    }
  }
  nn2 = nnchunk < P.nchunks ? load_desc(nnchunk) : nxt;
  if (P.ctr && tid == 0) {
    int64_t ch = P.nchunks;
    if (nnchunk < P.nchunks) {  // once the sequence has ended it stays ended
      if (gq >= 0) take_batch(gq, gcand);
      ch = grab();
    }
    s_idx[kpar] = ch;
  }
  if (bad) atomicOr(P.err, 1);
  __syncthreads();
  if (MAT == MAT_BLOCKS && P.bc) {
    for (int t = tid; t < nrows * GD; t += 256) {
      const int lr = t / GD, i = t % GD;
      if (!((s_rowbc[lr] >> i) & 1u)) continue;
      const int s = lds_find(cols, rowoff[lr], rowoff[lr + 1], (int32_t)(r0 + lr));
      if (s < 0) { atomicOr(P.err, 2); continue; }
      acc[s * BS2 + i * GD + i] = P.diag;
    }
    __syncthreads();
  }
  if (nchunk < P.nchunks) stage_meta(nxt);  // chunk k+1's metadata: every lane is past chunk k's items
  // Stream the chunk out: 16-B non-temporal stores (the matrix is written once and not re-read
  // by this launch, so it should not evict the records and dofmap the next chunks share).
  {
    const int64_t off = (b0 - abase) * BS2;  // first value, in doubles
    double* out = P.A.data + off;
    const int nv = nb * BS2;
    const int h = (int)(off & 1);  // one leading double when the chunk starts on an odd double
    if (h && tid == 0) __builtin_nontemporal_store(acc[0], out);
    const int np = (nv - h) >> 1;
    typedef double dv2 __attribute__((ext_vector_type(2)));
    dv2* out2 = reinterpret_cast<dv2*>(out + h);
    // a batch's LDS reads are issued together, then its stores (one LDS latency per batch,
    // not per store: the LDS is busy with other workgroups' atomics)
    constexpr int SU = kGatherStoreBatch;
    for (int t0 = tid; t0 < np; t0 += 256 * SU) {
      dv2 v[SU];
#pragma unroll
      for (int u = 0; u < SU; ++u) {
        const int t = t0 + 256 * u;
        if (t < np) {
          if (h) { v[u].x = acc[1 + 2 * t]; v[u].y = acc[2 + 2 * t]; }
          else v[u] = reinterpret_cast<const dv2*>(acc)[t];
        }
      }
#pragma unroll
      for (int u = 0; u < SU; ++u) {
        const int t = t0 + 256 * u;
        if (t < np) __builtin_nontemporal_store(v[u], out2 + t);
      }
      static_assert(SU == 4, "store_guard below");
      store_guard4(v[0], v[1], v[2], v[3]);
    }
    if (((nv - h) & 1) && tid == 0) __builtin_nontemporal_store(acc[nv - 1], out + nv - 1);
  }
  if (nchunk >= P.nchunks) break;
  __syncthreads();  // the store has read acc
  zero_acc(nxt);
  cur = nxt;
  nxt = nn2;
  nchunk = nnchunk;
  nnchunk = P.ctr ? (int64_t)__builtin_amdgcn_readfirstlane((int)s_idx[kpar])  // written before the items barrier
                  : chunk_of(vb + 3 * vstep);
  kpar ^= 1;
  vb += vstep;
  __syncthreads();
  }
}

// ------------------------------------------------------------------------------ store-decoupled gather
// k_gather_lin: the uniform-nu affine-simplex gather (MAT_LINU: configs A, C, E) with a positional
// plan, written so that a workgroup never waits for its own chunk stores. CDNA counts stores in
// vmcnt, and a wave's wait for a load also waits for every older vector-memory operation: in
// k_gather a chunk's item loads were issued after the previous chunk's stores, so every chunk's
// compute started only once those stores had drained (and its register spills waited vmcnt(0)).
// Here every vector-memory operation of the loop is unconditional and of a static count per lane
// (clamped addresses; lanes past a chunk's items or values store past the buffer range, which is
// dropped), so the compiler's vmcnt waits count exactly the operations issued after a load, and the
// loads of chunk k+1 (entries one chunk earlier still; FUSE: one stage more) are issued BEFORE chunk
// k's stores: the item phase of chunk k+1 waits for its own data only.
// Per chunk: items (LDS atomics; the packed reference-tensor block read one block ahead so the wait
// for it never includes the previous block's atomics) | barrier B1 | exchange every value of the
// chunk with zero into registers (each lane its own pairs: no second barrier), buffer stores
// (non-temporal, 16 B per lane, + the unpaired head / tail value) | barrier B3. The chunks come from
// 8 per-XCD counters (kLinCB; the counter's return is waited with the item loads). Dirichlet
// diagonals are set after the launch (k_bc_diag), items zero every constrained entry as in k_gather.
// Plans: <= NT items per chunk (fa_plan_gather caps a chunk at NT / NSPLIT adjacency entries and at
// lin_maxb blocks for these elements). DESIGN.md §3.2, §3.2b.
// chunk stores: non-temporal (plain stores measured 53.5 vs 49.8 ms on config E)
template <typename T>
__device__ __forceinline__ void lin_store(const T& v, T* p) {
  __builtin_nontemporal_store(v, p);
}

// chunk drain of k_gather_neo without the read / zero barrier (chunk_drain)
// Stream a chunk's nv accumulated values acc[h, h + nv) to out[0, nv) and leave the accumulator
// zero, after the items barrier. The values form 16-B pairs acc2[j], j < j1 = (h + nv + 1) / 2; pair
// j lands at out - h + 2j, 16-B aligned (out - h is). A lane reads, zeroes and stores its own pairs
// (SW per lane, j = tid + 256 u), so no barrier separates the reads from the zeroes; the partial
// pairs at the ends (head half when h = 1, tail half when h + nv is odd) are stored as single
// values by their owners. Every lane issues exactly SW + 2 stores (lanes without a pair or a half
// store to the scratch line `dump`): a static vector-memory count (see k_gather_lin).
// The stored values are left in v / hv / tv for the caller's keep_vgprs after its next barrier.
template <int SW, int NT = 256>
__device__ __forceinline__ void chunk_drain(double* acc, int h, int nv, double* out, int tid, fa_dv2 (&v)[SW],
                                            double& hv, double& tv) {
  typedef fa_dv2 dv2;
  typedef int v4i __attribute__((ext_vector_type(4)));
  typedef unsigned v2u __attribute__((ext_vector_type(2)));
  dv2* acc2 = reinterpret_cast<dv2*>(acc);
  const int j1 = (h + nv + 1) >> 1;
  const int jt = (h + nv - 1) >> 1;             // the pair holding the last value
  const bool tail_half = ((h + nv) & 1) != 0;  // ... alone
  // buffer stores over the chunk's 16-B-aligned span [out - h, out + nv): an offset past it is
  // dropped by the range check (no traffic), so every lane issues the same stores
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(out - h, 0, (h + nv) * 8, 0x00020000);
  constexpr int OOB = 0x40000000;
  constexpr int AUX = 2;  // nt
  hv = 0.0;
  tv = 0.0;
#pragma unroll
  for (int u = 0; u < SW; ++u) {
    const int j = tid + NT * u;
    const int jj = max(min(j, j1 - 1), 0);
    v[u] = acc2[jj];
    if (j < j1) acc2[jj] = dv2{0.0, 0.0};
    if (j == 0) hv = v[u].y;
    if (j == jt) tv = v[u].x;
    const bool full = j < j1 && !(j == 0 && h) && !(j == jt && tail_half);
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4i, v[u]), rs, full ? 16 * j : OOB, 0, AUX);
  }
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2u, hv), rs, (tid == 0 && h) ? 8 : OOB, 0, AUX);
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2u, tv), rs,
                                        (tid == (jt % NT) && tail_half && !(jt == 0 && h)) ? 8 * (h + nv - 1) : OOB, 0, AUX);
}
// k_gather_lin's drain as a function (k_gather_neo, round 5): after the items barrier, every value of
// the chunk is exchanged with zero into registers (ds_wrxchg_rtn_b64 at raised wave priority: the
// exchanges issue ahead of other workgroups' atomics), then stored with SW 16-B buffer stores per lane
// plus the unpaired head / tail value (lanes without one store past the descriptor's range: dropped).
// The caller's next barrier, then keep_vgprs(v, hv, tv), as in k_gather_lin.
template <int SW, int NT = 256>
__device__ __forceinline__ void xchg_drain(double* acc, int h, int nv, double* out, int tid, fa_dv2 (&v)[SW],
                                           double& hv, double& tv) {
  typedef int v4i __attribute__((ext_vector_type(4)));
  typedef unsigned v2u __attribute__((ext_vector_type(2)));
  const int np = (nv - h) >> 1;
  const bool tail = ((nv - h) & 1) != 0;
  hv = 0.0;
  tv = 0.0;
  __builtin_amdgcn_s_setprio(3);
  auto xchg = [&](double* p) -> double { return __hip_atomic_exchange(p, 0.0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); };
#pragma unroll
  for (int u = 0; u < SW; ++u) {
    v[u] = fa_dv2{0.0, 0.0};
    if (tid + NT * u < np) {
      double* pp = acc + 2 * (h + tid + NT * u);
      v[u] = fa_dv2{xchg(pp), xchg(pp + 1)};
    }
  }
  if (tid == 0 && h) hv = xchg(acc + 1);
  if (tid == 1 && tail) tv = xchg(acc + nv - 1 + h);
  __builtin_amdgcn_s_setprio(0);
  constexpr int OOB = 0x40000000, NTS = 2;  // nt
  const __amdgpu_buffer_rsrc_t rv = __builtin_amdgcn_make_buffer_rsrc(out, 0, 8 * nv, 0x00020000);
  const int base = 8 * h + 16 * tid, lim = np - tid;
#pragma unroll
  for (int u = 0; u < SW; ++u)
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4i, v[u]), rv, NT * u < lim ? base : OOB, 16 * NT * u, NTS);
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2u, hv), rv, (tid == 0 && h) ? 0 : OOB, 0, NTS);
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2u, tv), rv, (tid == 1 && tail) ? 8 * (nv - 1) : OOB, 0, NTS);
}
// An item's NBG slot words (u16) as packed pairs sl[t] = word 2t | word 2t+1 << 16. P2 simplices in
// column halves (NN 10, NSPLIT 2: 20 B per entry, part p at byte 10 p): three aligned dword loads at
// byte 8 p + {0, 4, 8}, shifted into place for the odd half (round 5; five u16 loads before: the
// gathers' loads are bound by instructions through the texture path, not bytes)
template <int NN, int NSPLIT, int NSL>
__device__ __forceinline__ void load_slot_words(const uint16_t* __restrict__ slots, int64_t e, int part,
                                                uint32_t (&sl)[NSL]) {
  constexpr int NBG = NN / NSPLIT;
  if constexpr (NN == 10 && NSPLIT == 2 && NSL == 3) {
    const uint32_t* w = reinterpret_cast<const uint32_t*>(slots + e * NN) + 2 * part;
    const uint32_t w0 = w[0], w1 = w[1], w2 = w[2];
    sl[0] = part ? __builtin_amdgcn_alignbit(w1, w0, 16) : w0;
    sl[1] = part ? __builtin_amdgcn_alignbit(w2, w1, 16) : w1;
    sl[2] = part ? (w2 >> 16) : (w2 & 0xFFFFu);
  } else {
    const uint16_t* sp = slots + e * NN + part * NBG;
#pragma unroll
    for (int t = 0; t < NSL; ++t)
      sl[t] = (uint32_t)sp[2 * t] | (2 * t + 1 < NBG ? (uint32_t)sp[2 * t + 1 < NBG ? 2 * t + 1 : 0] << 16 : 0u);
  }
}
constexpr int FA_LIN_FUSE = 1;  // P1 simplices (fa_assemble_matrix): records formed inside k_gather_lin
// 2^e for a normal exponent (|e| <= 1022), from its bits (no FP64 op: uniform e stays scalar)
__device__ __forceinline__ double pow2(int e) { return __hiloint2double((e + 1023) << 20, 0); }

// k_gather_lin's chunk schedule: a persistent grid of the resident workgroups pulls chunks from 8
// per-XCD counters (config E 38.3 vs 38.7 ms with ~32 chunks per workgroup in a static range; C 1.23
// vs 1.27 ms). Round 5: XCD x walks its own contiguous eighth [x per, (x + 1) per) of the visiting
// sequence (the plan's Morton order, fa_plan_locality, folded into the chunk arrays by
// lin_chunk_desc), so the chunks that share a cell's record run on one XCD, close in time, and
// the record is re-read from that XCD's L2. Dealing blocks of 16 row-order chunks round-robin to the
// XCDs (round 4) put the three lattice lines of a cell's rows on different XCDs: each record was
// fetched from beyond the L2 ~9 times (tools/r5/sim_l2.py: 8.7 modelled; 48.3 GB fetched per
// launch against ~17 GB read once, profiles/r4/final_pmc_E.txt); Morton per XCD models 1.6.

template <int GD, int NN, int NSPLIT, int NT = 256, bool FUSE = false, bool FIX = false>
__global__ __launch_bounds__(NT, NN == GD + 1 ? kLinWavesP1 : 4) void k_gather_lin(GatherArgs P, const uint32_t* __restrict__ zero32,
                                                        double* __restrict__ dump, int64_t per) {
  using R = Rec<GD, GD + 1, 1, MAT_LINU>;
  constexpr int BS2 = GD * GD;
  constexpr int NBG = NN / NSPLIT;
  constexpr int MAXB = lin_maxb(GD, NN);
  constexpr int NACC = MAXB * BS2 + 2;       // value p of a chunk at acc[p + h], h = its parity
  constexpr int NP2 = (NACC + 1) / 2;        // 16-B pairs of the accumulator
  constexpr int SW = (MAXB * BS2 / 2 + NT - 1) / NT;  // pair stores per lane per chunk
  constexpr int RL = R::SIZE;
  constexpr bool P1G = NN == GD + 1;
  static_assert(NN % NSPLIT == 0 && NN * GD <= 32 && RL % 2 == 0 && NN <= 63, "k_gather_lin: affine simplices");
  typedef double dv2 __attribute__((ext_vector_type(2)));
  __shared__ __attribute__((aligned(16))) double acc[2 * NP2];
  // the reference tensor, one packed integer block per (a, b) (pk_ahat: Ahat_ab = N_ab / D; the item
  // records are scaled by 1 / sqrt(D)); P1 simplices use none
  __shared__ uint64_t tab[P1G ? 1 : NN * NN];
  // FIX: per-block scale exponents of the chunks of each parity ([parity][chunk-relative block]: max
  // over the items adding into the block), round 6 (round 4-5: one exponent per chunk)
  __shared__ uint32_t s_bx[FIX ? 2 * MAXB : 1];
  constexpr int LOOK = FUSE ? 4 : 3;  // chunk descriptors in flight (d0 .. d[LOOK-1])
  constexpr int AHEAD = LOOK + 2;     // chunk ids fetched ahead of the chunk being gathered
  constexpr int RING = 8;
  __shared__ int32_t s_id[RING];      // chunk id of iteration m at s_id[m % RING]
  dv2* acc2 = reinterpret_cast<dv2*>(acc);
  const int tid = threadIdx.x;
  // Chunk schedule (kLinCB): the chunks being written at any time lie in one window of the rows, and
  // neighbouring chunks, which share cells, mostly run on one XCD (their records stay in its L2).
  // 32-bit chunk indices (the host checks nchunks < 2^30): fewer SGPRs in the loop
  const int xc = (int)(blockIdx.x % 8);  // the XCD under round-robin dispatch (speed only)
  // the j-th chunk of XCD counter x: position x * per + j of the visiting sequence (past the XCD's
  // eighth: nchunks, a descriptor of no entries)
  unsigned int* const lctr = reinterpret_cast<unsigned int*>(P.ctr) + 32 * xc;
  const unsigned int uper = (unsigned int)per, unc = (unsigned int)P.nchunks;
  auto chunk_of = [&](unsigned int j) -> int32_t {
    return (int32_t)(j < uper ? min((unsigned)xc * uper + j, unc) : unc);
  };
  if (tid == 0) {
    const unsigned int b = atomicAdd(lctr, (unsigned)AHEAD);
#pragma unroll
    for (int t = 0; t < AHEAD; ++t) s_id[t] = chunk_of(b + t);
  }
  __syncthreads();
  if constexpr (!P1G)
    for (int t = tid; t < NN * NN; t += NT) tab[t] = P.pk[t];
  for (int t = tid; t < NP2; t += NT) acc2[t] = dv2{0.0, 0.0};
  if constexpr (FIX)
    for (int t = tid; t < 2 * MAXB; t += NT) s_bx[t] = 0u;

  const int32_t* __restrict__ eadj = P.eadj;
  // a chunk: first block and adjacency entry, block and entry counts (< 2^31 each: fa_plan_gather's caps);
  // 6 SGPRs, and up to five in flight
  struct Desc { int64_t b0, a0; int32_t nb, na; };  // b0 relative to the window's first block
  // the workgroup's i-th chunk, clamped to its last: static loads of the per-launch chunk arrays
  // (chunk_b: first block relative to the window, chunk_a: first adjacency entry; lin_chunk_desc)
  // (the chunk of ring slot i; past the last chunk a descriptor of no entries and nb = -1)
  auto desc = [&](int i) -> Desc {
    const int raw = __builtin_amdgcn_readfirstlane(s_id[i % RING]);
    const bool ok = raw < (int)P.nchunks;
    const int c = ok ? raw : (int)P.nchunks - 1;
    const uint64_t n = (uint64_t)sload(P.chunk_a, (int64_t)P.nchunks + 1 + c);  // block count | entry count << 32
    return Desc{sload(P.chunk_b, c), sload(P.chunk_a, c), ok ? (int32_t)(uint32_t)n : -1, ok ? (int32_t)(n >> 32) : 0};
  };
  const int jit = tid / NSPLIT, part = tid % NSPLIT;
  // entry id (cell * NN + local row node) of this lane's item, clamped to a valid entry (chunk_a
  // holds each chunk's first entry clamped below the entry count)
  auto load_entry = [&](const Desc& d) -> int32_t { return eadj[d.a0 + min(jit, max(d.na - 1, 0))]; };
  // FUSE (P1 simplices, fa_assemble_matrix): no records kernel; an item loads its cell's vertex
  // coordinates, E and node bc bits (the vertex ids one chunk earlier still) and forms the uniform-nu
  // record in registers at the start of its chunk: one pipeline stage more (entries three chunks
  // ahead, vertex ids two, coordinates one), and no 80-B record written and re-read per cell
  static_assert(!FUSE || NN == GD + 1, "fused records: P1 simplices");
  constexpr int NV1 = GD + 1;
  struct Item {
    double r[RL];
    double x[FUSE ? NV1 : 1][GD];
    double E;
    uint32_t sl[(NBG + 1) / 2];  // the item's slot words, two 16-bit words per register
    uint32_t mask;
  };
  struct Vid { int32_t v[NV1]; };
  auto load_vid = [&](int32_t pflat) -> Vid {
    Vid w;
    const int32_t* g = P.M.geom + (int64_t)(pflat / NN) * NV1;
#pragma unroll
    for (int t = 0; t < NV1; ++t) w.v[t] = g[t];
    return w;
  };
  auto load_item = [&](const Desc& d, int32_t pflat, Item& it, const Vid& vd) {
    const int64_t c = pflat / NN;
    if constexpr (FUSE) {
      uint32_t m = 0u;
#pragma unroll
      for (int t = 0; t < NV1; ++t) {
        const fa_dv2* pn = reinterpret_cast<const fa_dv2*>(P.xpack + 4 * (int64_t)vd.v[t]);
        const fa_dv2 a = pn[0], b = pn[1];
        it.x[t][0] = a.x;
        it.x[t][1] = a.y;
        if constexpr (GD == 3) it.x[t][GD - 1] = b.x;
        m |= (uint32_t)__double_as_longlong(GD == 3 ? b.y : b.x) << (t * GD);
      }
      it.E = P.F.E[c];
      it.mask = m;
    } else {
      const dv2* rp = reinterpret_cast<const dv2*>(P.rec + c * RL);
#pragma unroll
      for (int k = 0; k < RL / 2; ++k) {
        const dv2 v = rp[k];
        it.r[2 * k] = v.x;
        it.r[2 * k + 1] = v.y;
      }
    }
    const int64_t e = d.a0 + min(jit, max(d.na - 1, 0));
    load_slot_words<NN, NSPLIT>(P.slots, e, part, it.sl);
    if constexpr (!FUSE) it.mask = rec_mask(it.r[GD * GD]);  // 0 without bcs (nothing was or-ed in)
  };
  // FUSE: the record (s Ji, sign of mu |J|) of the item's cell from its vertices (cell_record's
  // MAT_LINU branch on registers); table blocks: s Ji scaled by 1 / sqrt(D) of the packed table
  auto form_record = [&](Item& it) {
    if constexpr (!P1G) {
#pragma unroll
      for (int kk = 0; kk < BS2; ++kk) it.r[kk] *= P.pks;
    }
    if constexpr (FUSE) {
      double J[GD][GD], Ji[GD][GD];
#pragma unroll
      for (int kk = 0; kk < GD; ++kk)
#pragma unroll
        for (int i = 0; i < GD; ++i) J[i][kk] = it.x[kk + 1][i] - it.x[0][i];
      const double det = jac_inv<GD>(J, Ji);
      const double mu = it.E / (2.0 * (1.0 + P.F.nu));
      const double s2 = mu * fabs(det);
      const double sc = sqrt(fabs(s2));
#pragma unroll
      for (int i = 0; i < GD; ++i)
#pragma unroll
        for (int kk = 0; kk < GD; ++kk) it.r[i * GD + kk] = sc * Ji[i][kk];
      it.r[GD * GD] = s2 < 0.0 ? -1.0 : 1.0;
    }
  };
  // FIX (deterministic mode): every contribution v to block b of chunk k is added as the integer
  // round(v * 2^se_b) with ds_add_u64, so a block's sum is exact and independent of the order of
  // the adds; the drain converts it back (one rounding). se_b = 1072 - e_b with e_b the largest
  // biased exponent of the bounds fixc * rho^2 >= |block entry| of the items adding into block b,
  // so |v * 2^se| < 2^50 (the 1.5 * 2^52 rounding constant below is exact there) and up to 2^13
  // contributions never overflow. e_b is posted (ds_max_u32 into s_bx[k & 1][b], one per block of
  // the item) at the end of chunk k-1 from its prefetched items. Per BLOCK (round 6; the chunk-wide
  // exponent of rounds 4-5 summed a soft row beside stiff rows at the stiff rows' resolution, ~1e-13
  // x the stiffness contrast): every cell adding into block (a, b) holds node a, so the block's
  // scale is set by cells of its own row, and a row's error stays ~2^-50 of its own largest entry.
  auto bound_exp = [&](const Item& it, bool v) -> uint32_t {
    double rho = 0.0;
#pragma unroll
    for (int kk = 0; kk < BS2; ++kk) rho += fabs(it.r[kk]);
    const double m = P.fixc * rho * rho;
    return v ? (uint32_t)((uint64_t)__double_as_longlong(m) >> 52) & 0x7FFu : 0u;
  };
  auto post_bound = [&](const Item& it, const Desc& d, int par) {
    if (jit < d.na) {
      const uint32_t e = bound_exp(it, true);
#pragma unroll
      for (int bb = 0; bb < NBG; ++bb) {
        const int s = (int)((it.sl[bb / 2] >> (16 * (bb % 2))) & 1023u);
        if (s < d.nb) atomicMax(&s_bx[par * MAXB + s], e);
      }
    }
  };
  // 2^se of an exponent posted in s_bx (clamped: 2^(32 - se) stays finite)
  auto blk_scale = [&](uint32_t e) -> int { return max(-990, min(990, 1072 - (int)e)); };

  Desc d0 = desc(0), d1 = desc(1), d2 = desc(2), d3 = desc(3);
  int32_t pf0 = load_entry(d0), pf1 = load_entry(d1), pf2 = FUSE ? load_entry(d2) : 0;
  Item cur, nxt;
  Vid vid1{}, vid2{};
  if constexpr (FUSE) {
    const Vid vid0 = load_vid(pf0);
    vid1 = load_vid(pf1);
    load_item(d0, pf0, cur, vid0);
  } else {
    load_item(d0, pf0, cur, vid1);
  }
  int bad = 0;
  // the prologue's loads complete here (a builtin wait: the compiler's wait counting sees it, so the
  // loop's waits are not widened by pending prologue loads merged in at the loop head)
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
  __syncthreads();  // table and accumulator staged
  if constexpr (FIX) {  // chunk 0's scale
    form_record(cur);
    post_bound(cur, d0, 0);
    __syncthreads();
  }
  for (int k = 0; d0.nb >= 0; ++k) {
    // the id of chunk k + AHEAD
    unsigned int rn = 0u;
    // (atomicInc: the compiler's wave-aggregation of a uniform atomicAdd would wait for its return here)
    if (tid == 0) rn = atomicInc(lctr, 0xFFFFFFFFu);
    // L1: chunk k+2's entry ids; L2: chunk k+1's records / slots / masks (before chunk k's stores)
    // (FUSE: entries of chunk k+3, vertex ids of chunk k+2, coordinates of chunk k+1)
    int32_t pfn;
    if constexpr (FUSE) {
      pfn = load_entry(d3);
      vid2 = load_vid(pf2);
      load_item(d1, pf1, nxt, vid1);
    } else {
      pfn = load_entry(d2);
      load_item(d1, pf1, nxt, vid1);
    }
    const Desc d4 = desc(k + LOOK);
    if constexpr (!FIX) form_record(cur);  // FIX: formed at the end of the previous chunk (its bound)
    // items of chunk k
    const int64_t off = d0.b0 * BS2;
    const int h = (int)(off & 1);
    const int nb = d0.nb;
    const bool valid = jit < d0.na;
    // The LDS adds are issued by every lane (no branch): a lane without an item of this chunk (or, on
    // a broken pattern, with a slot past the chunk) adds zeros -- its record's s Ji zeroed -- to an
    // in-chunk slot of its own. Behind a branch the compiler could not count the outstanding LDS
    // operations and waited for each block's adds to complete (lgkmcnt(0)) before the next block's
    // prefetched table word.
    // (P2 / table blocks: config E 35.2 vs 36.0 ms. P1 simplices keep the branch: C 1.10 vs 1.11 ms,
    // their items are four table-free blocks)
    constexpr bool UNC = !P1G;
    int smax = 0;
#pragma unroll
    for (int bb = 0; bb < NBG; ++bb) smax = max(smax, (int)((cur.sl[bb / 2] >> (16 * (bb % 2))) & 1023u));
    bad |= valid && smax >= d0.nb;
    const bool eff = valid && smax < d0.nb;
    if constexpr (UNC) {
#pragma unroll
      for (int kk = 0; kk < BS2; ++kk) cur.r[kk] = eff ? cur.r[kk] : 0.0;
    }
    if (__any(eff)) {  // wave-uniform: a wave without items (a short chunk's last waves) skips them
      const int aloc = pf0 % NN;
      // the row's packed blocks: one ds_read_b64 per block (nine for a table of doubles)
      const uint64_t* Ah0 = tab + aloc * NN;
      const uint32_t rowm = (cur.mask >> (aloc * GD)) & ((1u << GD) - 1);
      const bool negw = __any(cur.r[BS2] < 0.0);  // wave-uniform: a cell with mu |J| < 0
      // P1 simplices (P1G): the scaled physical gradients are the rows of s Ji (node k >= 1) and minus
      // their sum (node 0), so K_ab = (1/GD!) [r g_a g_b^T + g_b g_a^T + (g_a . g_b) I] without the
      // reference-tensor table (no LDS reads; the column's gradient is selected from registers)
      double gA[GD];
      if constexpr (P1G) {
#pragma unroll
        for (int d = 0; d < GD; ++d) {
          double g0 = 0.0;
#pragma unroll
          for (int kk = 0; kk < GD; ++kk) g0 -= cur.r[kk * GD + d];
          gA[d] = g0;
#pragma unroll
          for (int kk = 0; kk < GD; ++kk) gA[d] = aloc == kk + 1 ? cur.r[kk * GD + d] : gA[d];
        }
      }
      // B_ab = r N_ab + N_ab^T (the integers of the packed block)
      auto unpack = [&](uint64_t q, double (&B)[BS2]) {
        constexpr int W = pk_width(GD), LO = pk_low(GD);
        const uint32_t q0 = (uint32_t)q, q1 = (uint32_t)(q >> 32);
        double N[BS2];
#pragma unroll
        for (int e = 0; e < BS2; ++e)
          N[e] = (double)(int)(e < LO ? __builtin_amdgcn_sbfe((int)q0, W * e, W) : __builtin_amdgcn_sbfe((int)q1, W * (e - LO), W));  // sbfe is typed unsigned
#pragma unroll
        for (int i = 0; i < GD; ++i)
#pragma unroll
          for (int k = 0; k < GD; ++k) B[i * GD + k] = fma(P.rlm, N[i * GD + k], N[k * GD + i]);
      };
      uint64_t qn = 0ull;
      if constexpr (!P1G) qn = Ah0[(cur.sl[0] >> 10) & 63u];
      // FIX: the blocks' scale exponents, read together before the adds (one LDS wait, not one per block)
      // (table blocks only: the fused P1 kernel has no registers to spare)
      uint32_t ex[FIX ? NBG : 1];
      if constexpr (FIX && !P1G) {
#pragma unroll
        for (int bb = 0; bb < NBG; ++bb) {
          const int sb = (int)((cur.sl[bb / 2] >> (16 * (bb % 2))) & 1023u);
          ex[bb] = s_bx[(k & 1) * MAXB + (eff ? sb : ((tid & 63) < nb ? (tid & 63) : 0))];
        }
      }
#pragma unroll
      for (int bb = 0; bb < NBG; ++bb) {
        const uint32_t slv = (cur.sl[bb / 2] >> (16 * (bb % 2))) & 0xFFFFu;
        const int s = (int)(slv & 1023u);
        const int b = (int)(slv >> 10);
        double G[GD][GD];
        if constexpr (P1G) {
          constexpr double cv = GD == 2 ? 0.5 : 1.0 / 6.0;  // reference simplex volume
          double gB[GD], dot = 0.0;
#pragma unroll
          for (int d = 0; d < GD; ++d) {
            double g0 = 0.0;
#pragma unroll
            for (int kk = 0; kk < GD; ++kk) g0 -= cur.r[kk * GD + d];
#pragma unroll
            for (int kk = 0; kk < GD; ++kk) g0 = b == kk + 1 ? cur.r[kk * GD + d] : g0;
            gB[d] = g0;
            dot = fma(gA[d], g0, dot);
          }
          const double ra = cv * P.rlm;
#pragma unroll
          for (int i = 0; i < GD; ++i)
#pragma unroll
            for (int kk = 0; kk < GD; ++kk) G[i][kk] = fma(ra * gA[i], gB[kk], cv * gB[i] * gA[kk]) + (i == kk ? cv * dot : 0.0);
        } else {
        double B[BS2];
        unpack(qn, B);
        if (bb + 1 < NBG)  // next block's table entry: issued before this block's atomics
          qn = Ah0[(cur.sl[(bb + 1) / 2] >> (16 * ((bb + 1) % 2) + 10)) & 63u];
        // G = (s Ji)^T B (s Ji), column by column; K = G + tr(G) / (1 + r) I
#pragma unroll
        for (int dd = 0; dd < GD; ++dd) {
          double T[GD];
#pragma unroll
          for (int i = 0; i < GD; ++i) {
            double t = B[i * GD] * cur.r[dd];
#pragma unroll
            for (int kk = 1; kk < GD; ++kk) t = fma(B[i * GD + kk], cur.r[kk * GD + dd], t);
            T[i] = t;
          }
#pragma unroll
          for (int e = 0; e < GD; ++e) {
            double g = cur.r[e] * T[0];
#pragma unroll
            for (int i = 1; i < GD; ++i) g = fma(cur.r[i * GD + e], T[i], g);
            G[e][dd] = g;
          }
        }
        double tr = G[0][0];
#pragma unroll
        for (int i = 1; i < GD; ++i) tr += G[i][i];
        tr *= P.trc;
#pragma unroll
        for (int i = 0; i < GD; ++i) G[i][i] += tr;
        }
        if (negw) {
          const double sg = rec_sign(cur.r[BS2]);
#pragma unroll
          for (int i = 0; i < GD; ++i)
#pragma unroll
            for (int kk = 0; kk < GD; ++kk) G[i][kk] *= sg;
        }
        const uint32_t colm = (cur.mask >> (b * GD)) & ((1u << GD) - 1);
        if (__any((rowm | colm) != 0u)) {
#pragma unroll
          for (int i = 0; i < GD; ++i)
#pragma unroll
            for (int kk = 0; kk < GD; ++kk)
              if (((rowm >> i) | (colm >> kk)) & 1u) G[i][kk] = 0.0;
        }
        if (UNC || eff) {
          const int sd = eff ? s : ((tid & 63) < nb ? (tid & 63) : 0);  // (zeros) distinct slots
          double* ap = acc + h + sd * BS2;
          if constexpr (FIX) {
            const double S = pow2(blk_scale(P1G ? s_bx[(k & 1) * MAXB + sd] : ex[bb]));  // the block's scale
#pragma unroll
            for (int i = 0; i < GD; ++i)
#pragma unroll
              for (int kk = 0; kk < GD; ++kk) {
                // round(v * 2^se): v * 2^se + 1.5 * 2^52 has a unit ulp for |v * 2^se| < 2^51, and its
                // bits minus those of 1.5 * 2^52 are that integer (two's complement)
                const double t = fma(G[i][kk], S, 0x1.8p52);
                const unsigned long long q = (unsigned long long)__double_as_longlong(t) - 0x4338000000000000ull;
                atomicAdd(reinterpret_cast<unsigned long long*>(ap + i * GD + kk), q);
              }
          } else {
#pragma unroll
            for (int i = 0; i < GD; ++i)
#pragma unroll
              for (int kk = 0; kk < GD; ++kk) atomicAdd(ap + i * GD + kk, G[i][kk]);
          }
        }
      }
    }
    __syncthreads();  // B1: the chunk is accumulated
    // the exchanges at raised wave priority: they issue ahead of other workgroups' atomics on the
    // CU (E 37.4 -> 36.6 ms, C 1.15 -> 1.13 ms; over B1 .. B3: 36.7 / 1.12-1.13)
    __builtin_amdgcn_s_setprio(3);
    // read the chunk into registers and leave the accumulator zero: pairs t (value 2t + h .. 2t + 1 + h
    // at acc2[t + h]) by lane t % NT, the unpaired head (acc[1] when h = 1) by lane 0, the unpaired
    // tail by lane 1; no other lane touches them, so no barrier separates the reads from the zeroes
    // (the other halves of the head / tail pairs are never written)
    const int nv = nb * BS2;
    const int np = (nv - h) >> 1;
    const bool tail = ((nv - h) & 1) != 0;
    dv2 v[SW];
    double hv = 0.0, tv = 0.0;
    {  // ds_wrxchg_rtn_b64: 2 x 6.4 LDS clocks per 16 B against 4.1 + 13.0 for a 16-B read and zero write
      auto xchg = [&](double* p) -> double {
        return __hip_atomic_exchange(p, 0.0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      };
#pragma unroll
      for (int u = 0; u < SW; ++u) {
        v[u] = dv2{0.0, 0.0};
        if (tid + NT * u < np) {
          double* pp = acc + 2 * (h + tid + NT * u);
          v[u] = dv2{xchg(pp), xchg(pp + 1)};
        }
      }
      if (tid == 0 && h) hv = xchg(acc + 1);
      if (tid == 1 && tail) tv = xchg(acc + nv - 1 + h);
    }
    __builtin_amdgcn_s_setprio(0);
    if constexpr (FIX) {  // the integer sums back to doubles: (hi 2^32 + lo) 2^-se_b, one rounding
      const uint32_t* bx = s_bx + (k & 1) * MAXB;
      auto tod = [&](double x, int p) -> double {  // value p of the chunk (block p / BS2)
        const int se = blk_scale(bx[min(max(p, 0) / BS2, MAXB - 1)]);
        const long long q = __double_as_longlong(x);
        return fma((double)(int)(q >> 32), pow2(32 - se), (double)(unsigned)q * pow2(-se));
      };
#pragma unroll
      for (int u = 0; u < SW; ++u) {
        const int p = 2 * (tid + NT * u) + h;  // pair t holds values 2t + h, 2t + h + 1
        v[u] = dv2{tod(v[u].x, p), tod(v[u].y, p + 1)};
      }
      hv = tod(hv, 0);
      tv = tod(tv, nv - 1);
    }
    // stores: SW pair stores + the head and the tail value on every lane (a static count: see above),
    // as buffer stores over the chunk's values; a lane without a pair (or the head / tail value)
    // stores at an offset past the range, which the range check drops (no memory traffic)
    {
      typedef int v4i __attribute__((ext_vector_type(4)));
      typedef unsigned v2u __attribute__((ext_vector_type(2)));
      constexpr int OOB = 0x40000000, NTS = 2;  // nt
      // one descriptor over the chunk's nv values; pair t at value h + 2t (16-B aligned)
      const __amdgpu_buffer_rsrc_t rv = __builtin_amdgcn_make_buffer_rsrc(P.A.data + off, 0, 8 * nv, 0x00020000);
      const int base = 8 * h + 16 * tid, lim = np - tid;  // pair tid + NT u: byte base + 16 NT u
#pragma unroll
      for (int u = 0; u < SW; ++u)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4i, v[u]), rv, NT * u < lim ? base : OOB, 16 * NT * u,
                                               NTS);
      __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2u, hv), rv, (tid == 0 && h) ? 0 : OOB, 0, NTS);
      __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2u, tv), rv, (tid == 1 && tail) ? 8 * (nv - 1) : OOB, 0, NTS);
    }
    if constexpr (FIX) {  // chunk k+1's scale from its prefetched items (records formed here for FUSE)
      form_record(nxt);
      post_bound(nxt, d1, (int)((k + 1) & 1));
    }
    __syncthreads();  // B3: the accumulator is clean for the next chunk's atomics
    keep_vgprs(v, hv, tv);
    if constexpr (FIX)  // chunk k's exponents are read; parity k & 1 is next posted at the end of chunk k + 1
      for (int t = tid; t < nb; t += NT) s_bx[(k & 1) * MAXB + t] = 0u;
    // chunk k + AHEAD's id, read at iteration k + AHEAD - LOOK = k + 2 (after B1 of k + 1); written
    // here, where the wait for it is the one for chunk k+1's item loads (issued after it)
    if (tid == 0) s_id[(k + AHEAD) % RING] = chunk_of(rn);
    // rotate the pipeline
    d0 = d1;
    d1 = d2;
    if constexpr (FUSE) {
      d2 = d3;
      d3 = d4;
      pf0 = pf1;
      pf1 = pf2;
      pf2 = pfn;
      vid1 = vid2;
    } else {
      d2 = d4;
      pf0 = pf1;
      pf1 = pfn;
    }
    cur = nxt;
  }
  if (bad) atomicOr(P.err, 1);
}

// ------------------------------------------------------------------------------ neo-Hookean M gather
// k_gather_neo: the neo-Hookean tangent (FA_NEO_HOOKEAN) on affine simplices with k_gather_lin's
// store-decoupled schedule. With g_b = Ji^T dphi_b (dphi_b the reference gradient at point q) the
// block is
//   K_ab = sum_q [ s_c (M_q dphi_a)(M_q dphi_b)^T - rho_q (M_q dphi_b)(M_q dphi_a)^T ]
//          + (sum_jl S_jl T_ab[j][l]) I,
// M_q = sqrt(w_q |J|) C'_q Ji^T (C'_q = sqrt|c2| cof F_q, the scaled cofactor of FA_NEO_SREC),
// S = mu |J| Ji Ji^T and T_ab[j][l] = sum_q w_q dphi_a[j] dphi_b[l] (the reference tensor of the
// mu (g_a . g_b) I term, identical to the per-point sum: the same rule). Per block and point:
// 3 LDS reads, V = M_q dphi_b (9 FMA), K += W V^T - V Z^T (18 FMA) with W = s_c M_q dphi_a and
// Z = rho_q M_q dphi_a formed once per item; the mu term is 6 table reads and 6 FMA per block
// (the per-point C g_b, g_b and dot of k_gather's neo items cost 42 FMA per block and point).
// Records (NeoM, 64-cell tiles as FA_NEO_TILE): head S (upper triangle), s_c | per point M_q, rho_q.
template <int GD, int NQ>
struct NeoM {
  static constexpr int NT = GD * (GD + 1) / 2;         // S / T entries: 00 11 (22) 01 (02 12)
  static constexpr int HEAD = (NT + 1 + 1) & ~1;       // S, s_c (even)
  static constexpr int PT = (GD * GD + 1 + 1) & ~1;    // M_q, rho_q (even)
  static constexpr int SIZE = HEAD + NQ * PT;
  __host__ __device__ static constexpr int64_t head(int64_t c) { return (c >> 6) * (64 * SIZE) + (c & 63) * HEAD; }
  __host__ __device__ static constexpr int64_t point(int64_t c, int q) {
    return (c >> 6) * (64 * SIZE) + 64 * HEAD + q * (64 * PT) + (c & 63) * PT;
  }
  __host__ __device__ static constexpr int64_t count(int64_t nc) { return (nc + 63) / 64 * 64 * SIZE; }
};
// symmetric-pair index of NeoM's S / T entries: (j, l) -> 0..NT-1 (diagonal first)
template <int GD>
__host__ __device__ constexpr int sym_pair(int j, int l) {
  return j == l ? j : (GD == 2 ? 2 : (j + l == 1 ? 3 : (j + l == 2 ? 4 : 5)));
}

// NeoM records, one wave per 64-cell tile (lane = cell), each block of the tile staged in
// wave-private LDS and stored as one contiguous run (as k_neo_records_tiled). 3 waves / SIMD (168
// VGPRs, 2 spilled outside the point loop): E-neo 64.3 vs 65.2 ms at 2 (195 VGPRs), 68.4 at 4
template <int GD, int NN, int NQ>
__global__ __launch_bounds__(256, 3) void k_neo_records_m(MeshView M, FormView F, const double* __restrict__ tab,
                                                       const int8_t* __restrict__ bc, double* __restrict__ rec,
                                                       uint32_t* __restrict__ bcmask) {
  using R = NeoM<GD, NQ>;
  static_assert(NN * GD <= 32, "bc mask holds 32 dofs");
  constexpr int N = GD * GD, HD = R::HEAD, PT = R::PT;
  constexpr int BUF = 64 * (HD > PT ? HD : PT);
  __shared__ __attribute__((aligned(16))) double sbuf[4][BUF];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  double* sb = sbuf[wave];
  auto wave_sync = [] {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  };
  auto flush = [&](double* dst, int n) {  // sb[0, n) -> dst, n even, dst 16-B aligned
    wave_sync();
    const fa_dv2* s2 = reinterpret_cast<const fa_dv2*>(sb);
    fa_dv2* d2 = reinterpret_cast<fa_dv2*>(dst);
    for (int t = lane; t < n / 2; t += 64) {
      const fa_dv2 v = s2[t];
      d2[t] = v;
      store_guard1(v);
    }
    wave_sync();
  };
  const int64_t ntiles = (M.ncells + 63) / 64;
  for (int64_t tile = blockIdx.x * 4 + wave; tile < ntiles; tile += (int64_t)gridDim.x * 4) {
    const int64_t c0 = tile * 64 + lane;
    const bool valid = c0 < M.ncells;
    const int64_t c = valid ? c0 : M.ncells - 1;  // lanes past the end fill the tile's padding
    double* tb = rec + tile * (64 * R::SIZE);
    double Ji[GD][GD];
    const double det = fabs(simplex_geometry<GD>(M, c, Ji));
    double lam, mu;
    cell_lame(F, c, lam, mu);
    const double sgn = lam > 0.0 ? 1.0 : (lam < 0.0 ? -1.0 : 0.0);  // sign of W_JJ + W_J/J = lam / J^2
#pragma unroll
    for (int j = 0; j < GD; ++j)
#pragma unroll
      for (int l = j; l < GD; ++l) {
        double s = 0.0;
#pragma unroll
        for (int d = 0; d < GD; ++d) s = fma(Ji[j][d], Ji[l][d], s);
        sb[lane * HD + sym_pair<GD>(j, l)] = mu * det * s;
      }
    sb[lane * HD + R::NT] = sgn;
#pragma unroll
    for (int t = R::NT + 1; t < HD; ++t) sb[lane * HD + t] = 0.0;
    flush(tb, 64 * HD);
    const int32_t* cn = M.cells + c * NN;
    // the cell's nodal displacements once (not per point): F_q = I + (sum_b u_b dphi_b(q)^T) Ji
    double ue[NN][GD];
#pragma unroll
    for (int b = 0; b < NN; ++b) {
      const int64_t n = cn[b];
#pragma unroll
      for (int i = 0; i < GD; ++i) ue[b][i] = F.u[n * GD + i];
    }
    for (int q = 0; q < NQ; ++q) {
      double Gr[GD][GD];
#pragma unroll
      for (int i = 0; i < GD; ++i)
#pragma unroll
        for (int k = 0; k < GD; ++k) Gr[i][k] = 0.0;
      const double* dq = tab + NQ + q * NN * GD;
#pragma unroll
      for (int b = 0; b < NN; ++b)
#pragma unroll
        for (int i = 0; i < GD; ++i)
#pragma unroll
          for (int k = 0; k < GD; ++k) Gr[i][k] = fma(ue[b][i], dq[b * GD + k], Gr[i][k]);
      double Fq[N];
#pragma unroll
      for (int i = 0; i < GD; ++i)
#pragma unroll
        for (int d = 0; d < GD; ++d) {
          double f = i == d ? 1.0 : 0.0;
#pragma unroll
          for (int k = 0; k < GD; ++k) f = fma(Gr[i][k], Ji[k][d], f);
          Fq[i * GD + d] = f;
        }
      double I1 = GD == 2 ? 1.0 : 0.0, J;
#pragma unroll
      for (int m = 0; m < N; ++m) I1 = fma(Fq[m], Fq[m], I1);
      if constexpr (GD == 2) J = Fq[0] * Fq[3] - Fq[1] * Fq[2];
      else J = Fq[0] * (Fq[4] * Fq[8] - Fq[5] * Fq[7]) - Fq[1] * (Fq[3] * Fq[8] - Fq[5] * Fq[6]) +
               Fq[2] * (Fq[3] * Fq[7] - Fq[4] * Fq[6]);
      double co[5];
      neo_energy_coeffs(I1, J, lam, mu, co);
      double Cm[GD][GD];
      cofactor<GD>(Fq, Cm);
      const double a2 = fabs(co[2]);
      const double sc = (sgn != 0.0 ? sqrt(a2) : 1.0) * sqrt(tab[q] * det);
      const double rho = sgn != 0.0 ? co[3] / a2 : co[3];
#pragma unroll
      for (int i = 0; i < GD; ++i)
#pragma unroll
        for (int k = 0; k < GD; ++k) {
          double m = 0.0;
#pragma unroll
          for (int d = 0; d < GD; ++d) m = fma(Cm[i][d], Ji[k][d], m);
          sb[lane * PT + i * GD + k] = sc * m;
        }
      sb[lane * PT + N] = rho;
#pragma unroll
      for (int t = N + 1; t < PT; ++t) sb[lane * PT + t] = 0.0;
      flush(tb + 64 * HD + q * (64 * PT), 64 * PT);
    }
    if (bcmask && valid) {
      uint32_t m = 0;
#pragma unroll
      for (int b = 0; b < NN; ++b) {
        const int64_t n = cn[b];
#pragma unroll
        for (int j = 0; j < GD; ++j) m |= (bc[n * GD + j] ? 1u : 0u) << (b * GD + j);
      }
      bcmask[c] = m;
    }
  }
}

// 2 waves / SIMD (215 VGPRs, no spills in the item loop; 3 waves measured slower: spilled records)
template <int GD, int NN, int NQ, int NSPLIT>
__global__ __launch_bounds__(256, 2) void k_gather_neo(GatherArgs P, const uint32_t* __restrict__ zero32,
                                                       double* __restrict__ dump, int64_t per) {
  using R = NeoM<GD, NQ>;
  constexpr int NTH = 256;  // threads: 256 items
  constexpr int BS2 = GD * GD, NT = R::NT, NQL = NQ;
  constexpr int NBG = NN / NSPLIT;
  constexpr int MAXB = gather_maxb(true, BS2);
  constexpr int NACC = MAXB * BS2 + 2;
  constexpr int NP2 = (NACC + 1) / 2;
  // pairs per lane of chunk_drain: a chunk spans up to (h + MAXB * BS2 + 1) / 2 16-B pairs
  constexpr int SW = (MAXB * BS2 / 2 + 1 + NTH - 1) / NTH;
  static_assert(SW * NTH >= (MAXB * BS2 + 1) / 2 + 1, "chunk_drain covers every pair");
  static_assert(NN % NSPLIT == 0 && NN * GD <= 32 && NN <= 63 && MAXB < 1024,
                "k_gather_neo: affine simplices");
  typedef double dv2 __attribute__((ext_vector_type(2)));
  __shared__ __attribute__((aligned(16))) double acc[2 * NP2];
  __shared__ __attribute__((aligned(16))) double s_phi[NN * NQ * GD];  // [b][q][k]: a column's gradients at every point, contiguous
  __shared__ __attribute__((aligned(16))) double s_T[NN * NN * NT];    // [a][b][t]
  dv2* acc2 = reinterpret_cast<dv2*>(acc);
  const int tid = threadIdx.x;
  // chunk schedule of k_gather_lin (round 5): the resident grid pulls chunks from 8 per-XCD counters,
  // XCD x walking its eighth of the plan's visiting sequence (lin_chunk_desc's arrays), ids fetched
  // AHEAD iterations ahead through an LDS ring. (Round 4: ~128 chunks per workgroup in a static
  // strided range of the Morton order; consecutive iterations were G chunks apart, so a 384-B record
  // was fetched from beyond the L2 ~5.5 times: 106.5 GB per launch, profiles/r4/final_pmc_Eneo.txt.)
  constexpr int LOOK = 3, AHEAD = LOOK + 2, RING = 8;
  __shared__ int32_t s_id[RING];
  const int xc = (int)(blockIdx.x % 8);
  unsigned int* const lctr = reinterpret_cast<unsigned int*>(P.ctr) + 32 * xc;
  const unsigned int uper = (unsigned int)per, unc = (unsigned int)P.nchunks;
  auto chunk_of = [&](unsigned int j) -> int32_t {
    return (int32_t)(j < uper ? min((unsigned)xc * uper + j, unc) : unc);
  };
  if (tid == 0) {
    const unsigned int b = atomicAdd(lctr, (unsigned)AHEAD);
#pragma unroll
    for (int t = 0; t < AHEAD; ++t) s_id[t] = chunk_of(b + t);
  }
  const double* wq = P.tab;
  const double* dphi = P.tab + NQ;  // [q][b][k]
  for (int t = tid; t < NN * NQ * GD; t += NTH) {
    const int b = t / (NQ * GD), q = (t / GD) % NQ, k = t % GD;
    s_phi[t] = dphi[(q * NN + b) * GD + k];
  }
  for (int t = tid; t < NN * NN; t += NTH) {
    const int a = t / NN, b = t % NN;
    double Ah[GD][GD];
#pragma unroll
    for (int j = 0; j < GD; ++j)
#pragma unroll
      for (int l = 0; l < GD; ++l) Ah[j][l] = 0.0;
    for (int q = 0; q < NQ; ++q)
#pragma unroll
      for (int j = 0; j < GD; ++j)
#pragma unroll
        for (int l = 0; l < GD; ++l) Ah[j][l] = fma(wq[q] * dphi[(q * NN + a) * GD + j], dphi[(q * NN + b) * GD + l], Ah[j][l]);
#pragma unroll
    for (int j = 0; j < GD; ++j)
#pragma unroll
      for (int l = j; l < GD; ++l) s_T[t * NT + sym_pair<GD>(j, l)] = j == l ? Ah[j][j] : Ah[j][l] + Ah[l][j];
  }
  for (int t = tid; t < NP2; t += NTH) acc2[t] = dv2{0.0, 0.0};

  const int32_t* __restrict__ eadj = P.eadj;
  const uint32_t* __restrict__ mk = P.bcmask ? P.bcmask : zero32;
  const uint32_t mkmul = P.bcmask ? 1u : 0u;
  // a chunk (lin_chunk_desc): first block relative to the window, first adjacency entry (clamped
  // below the entry count), block and entry counts; past the XCD's eighth nb = -1 and no entries
  struct Desc { int64_t b0, a0; int32_t nb, na; };
  __syncthreads();  // s_id staged
  auto desc = [&](int i) -> Desc {
    const int raw = __builtin_amdgcn_readfirstlane(s_id[i % RING]);
    const bool ok = raw < (int)P.nchunks;
    const int c = ok ? raw : (int)P.nchunks - 1;
    const uint64_t n = (uint64_t)sload(P.chunk_a, (int64_t)P.nchunks + 1 + c);  // block count | entry count << 32
    return Desc{sload(P.chunk_b, c), sload(P.chunk_a, c), ok ? (int32_t)(uint32_t)n : -1, ok ? (int32_t)(n >> 32) : 0};
  };
  const int item = tid;
  const int jit = item / NSPLIT, part = item % NSPLIT;
  auto entry_of = [&](const Desc& d) -> int64_t { return d.a0 + min(jit, max(d.na - 1, 0)); };
  auto load_entry = [&](const Desc& d) -> int32_t { return eadj[entry_of(d)]; };
  // the head's S and s_c (NT + 1 values; its padding is not loaded); slots two per register
  constexpr int HL = NT + 1, NSL = (NBG + 1) / 2;
  struct Item { double hd[HL]; double pt[NQL][R::PT]; uint32_t sl[NSL]; uint32_t mask; };
  auto load_item = [&](const Desc& d, int32_t pflat, Item& it) {
    const int64_t c = pflat / NN;
    const double* hq = P.rec + R::head(c);
    const dv2* hp = reinterpret_cast<const dv2*>(hq);
#pragma unroll
    for (int k = 0; k < HL / 2; ++k) {
      const dv2 v = hp[k];
      it.hd[2 * k] = v.x;
      it.hd[2 * k + 1] = v.y;
    }
    if constexpr (HL % 2) it.hd[HL - 1] = hq[HL - 1];
#pragma unroll
    for (int ql = 0; ql < NQL; ++ql) {
      const dv2* pp = reinterpret_cast<const dv2*>(P.rec + R::point(c, ql));
#pragma unroll
      for (int k = 0; k < R::PT / 2; ++k) {
        const dv2 v = pp[k];
        it.pt[ql][2 * k] = v.x;
        it.pt[ql][2 * k + 1] = v.y;
      }
    }
    load_slot_words<NN, NSPLIT>(P.slots, entry_of(d), part, it.sl);
    it.mask = mk[c * mkmul] * mkmul;
  };
  Desc d0 = desc(0), d1 = desc(1), d2 = desc(2);
  int32_t pf0 = load_entry(d0), pf1 = load_entry(d1);
  Item cur;
  load_item(d0, pf0, cur);
  int bad = 0;
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): the prologue's loads (see k_gather_lin)
  __syncthreads();                     // tables and accumulator staged
  for (int k = 0; d0.nb >= 0; ++k) {
    unsigned int rn = 0u;  // the id of chunk k + AHEAD (atomicInc: see k_gather_lin)
    if (tid == 0) rn = atomicInc(lctr, 0xFFFFFFFFu);
    const int32_t pf2 = load_entry(d2);  // chunk k+2's entry ids
    const Desc d3 = desc(k + LOOK);
    const int64_t off = d0.b0 * BS2;
    const int h = (int)(off & 1);
    const int nb = d0.nb;
    const bool valid = jit < d0.na;
    {
      const int aloc = pf0 % NN;
      const uint32_t rowm = (cur.mask >> (aloc * GD)) & ((1u << GD) - 1);
      // The LDS adds are issued by every lane (no branch): a lane without an item of this chunk (or,
      // on a broken pattern, with a slot past the chunk) adds zeros to an in-chunk slot of its own.
      // Behind a branch the compiler could not count the outstanding LDS operations and waited for
      // each block's adds to complete (lgkmcnt(0)) before the next block's prefetched table values.
      int smax = 0;
#pragma unroll
      for (int bb = 0; bb < NBG; ++bb) smax = max(smax, (int)((cur.sl[bb / 2] >> (16 * (bb % 2))) & 1023u));
      bad |= valid && smax >= nb;
      const bool eff = valid && smax < nb;
      if (__any(eff)) {  // wave-uniform: a wave without items skips them
      const double sc = eff ? cur.hd[NT] : 0.0;
#pragma unroll
      for (int t = 0; t < NT; ++t) cur.hd[t] = eff ? cur.hd[t] : 0.0;
      // per point: U = M_q dphi_a, W = s_c U, Z = rho_q U
      double W[NQL][GD], Z[NQL][GD];
#pragma unroll
      for (int ql = 0; ql < NQL; ++ql) {
        const int q = ql;
        double pa[GD];
#pragma unroll
        for (int kk = 0; kk < GD; ++kk) pa[kk] = s_phi[(aloc * NQ + q) * GD + kk];
#pragma unroll
        for (int i = 0; i < GD; ++i) {
          double u = cur.pt[ql][i * GD] * pa[0];
#pragma unroll
          for (int kk = 1; kk < GD; ++kk) u = fma(cur.pt[ql][i * GD + kk], pa[kk], u);
          W[ql][i] = sc * u;
          Z[ql][i] = (eff ? cur.pt[ql][BS2] : 0.0) * u;
        }
      }
      // the column's table values (its gradients at every point, its mu-term block) of block bb + 1
      // are read into registers while block bb computes: the reads' LDS latency is not exposed per
      // point (round 4 read them through a volatile pointer right before each use: 3-4 dependent
      // waits per point, 5 blocks per item)
      const double* Ta = s_T + aloc * NN * NT;
      auto col_of = [&](int bb) -> uint32_t { return (cur.sl[bb / 2] >> (16 * (bb % 2))) & 0xFFFFu; };
      // (the mu-term block is read at the top of its own block: it is needed last)
      struct Col { double ph[NQL * GD]; };
      auto load_col = [&](int b, Col& c) {
#pragma unroll
        for (int u = 0; u < NQL * GD; ++u) c.ph[u] = s_phi[b * NQ * GD + u];
      };
      Col cn;
      load_col((int)(col_of(0) >> 10), cn);
#pragma unroll
      for (int bb = 0; bb < NBG; ++bb) {
        const uint32_t slv = col_of(bb);
        const int s = (int)(slv & 1023u);
        const int b = (int)(slv >> 10);
        const Col cc = cn;
        double tt[NT];
#pragma unroll
        for (int u = 0; u < NT; ++u) tt[u] = Ta[b * NT + u];
        if (bb + 1 < NBG) load_col((int)(col_of(bb + 1) >> 10), cn);
        double K[GD][GD];
#pragma unroll
        for (int i = 0; i < GD; ++i)
#pragma unroll
          for (int kk = 0; kk < GD; ++kk) K[i][kk] = 0.0;
#pragma unroll
        for (int ql = 0; ql < NQL; ++ql) {
          double V[GD];
#pragma unroll
          for (int i = 0; i < GD; ++i) {
            double v = cur.pt[ql][i * GD] * cc.ph[ql * GD];
#pragma unroll
            for (int kk = 1; kk < GD; ++kk) v = fma(cur.pt[ql][i * GD + kk], cc.ph[ql * GD + kk], v);
            V[i] = v;
          }
#pragma unroll
          for (int i = 0; i < GD; ++i)
#pragma unroll
            for (int kk = 0; kk < GD; ++kk) K[i][kk] = fma(W[ql][i], V[kk], fma(-V[i], Z[ql][kk], K[i][kk]));
        }
        {
          double dot = 0.0;
#pragma unroll
          for (int t = 0; t < NT; ++t) dot = fma(cur.hd[t], tt[t], dot);
#pragma unroll
          for (int i = 0; i < GD; ++i) K[i][i] += dot;
        }
        const uint32_t colm = (cur.mask >> (b * GD)) & ((1u << GD) - 1);
        if (__any((rowm | colm) != 0u)) {
#pragma unroll
          for (int i = 0; i < GD; ++i)
#pragma unroll
            for (int kk = 0; kk < GD; ++kk)
              if (((rowm >> i) | (colm >> kk)) & 1u) K[i][kk] = 0.0;
        }
        const int se = eff ? s : ((tid & 63) < nb ? (tid & 63) : 0);  // (zeros) distinct slots
        {
          double* ap = acc + h + se * BS2;
#pragma unroll
          for (int i = 0; i < GD; ++i)
#pragma unroll
            for (int kk = 0; kk < GD; ++kk) atomicAdd(ap + i * GD + kk, K[i][kk]);
        }
      }
      }
    }
    // chunk k+1's records / slots / masks: the item registers are dead here, and these loads are
    // issued before chunk k's stores (their wait at chunk k+1 does not include the stores)
    load_item(d1, pf1, cur);
    __syncthreads();  // B1: the chunk is accumulated
    fa_dv2 dv[SW];
    double dh, dt;
    xchg_drain<SW, NTH>(acc, h, nb * BS2, P.A.data + off, tid, dv, dh, dt);
    __syncthreads();  // B3: the accumulator is clean for the next chunk's atomics
    keep_vgprs(dv, dh, dt);
    // chunk k + AHEAD's id, read at iteration k + AHEAD - LOOK (after later barriers)
    if (tid == 0) s_id[(k + AHEAD) % RING] = chunk_of(rn);
    d0 = d1;
    d1 = d2;
    d2 = d3;
    pf0 = pf1;
    pf1 = pf2;
  }
  if (bad) atomicOr(P.err, 1);
}

// ------------------------------------------------------------------------------ block-owner gather
// k_gather_own: the uniform-nu affine-simplex gather (MAT_LINU) without per-contribution LDS
// atomics. The contribution plan (fa_plan_contrib) lists, per chunk, every (cell, row node a,
// column node b) contribution sorted by destination block and cut into 256 equal lane segments
// (K per lane). A lane sums its segment's contributions to one block in registers and writes the
// block once, with a plain LDS store, at the block's last contribution; a lane whose segment ends
// inside a block adds that partial sum with one LDS atomic after a barrier (about half of the
// lanes, once per chunk). The chunk's distinct cells' records are staged in LDS once per chunk
// (one 80-B load per cell instead of one per item), the reference-tensor table B_ab sits in LDS.
// Output: the chunk is streamed to HBM with coalesced 16-B stores, exactly as k_gather does.
constexpr int FA_OWN_LDS = 28672;  // output staging bytes per workgroup
constexpr int FA_OWN_CCAP = 256;  // distinct cells (and adjacency entries) per chunk of a contribution plan (8-bit slots);
                         // config C 2.87 ms at 128 -> 2.07 at 256, A 0.155 -> 0.136 ms
__host__ __device__ constexpr int own_maxb(int bs2) { return FA_OWN_LDS / (8 * bs2) < 1023 ? FA_OWN_LDS / (8 * bs2) : 1023; }
// contribution word (u16): bits 0-7 cell slot, 8-14 a * NN + b (127: padding), 15 last of its block
constexpr uint32_t kOwnPad = 0x7F00u;
constexpr uint32_t kOwnIdle = 0xFFFFu;  // lane start of a lane with no contribution

template <int GD, int NN>
__global__ __launch_bounds__(256, 3) void k_gather_own(GatherArgs P) {
  using R = Rec<GD, GD + 1, 1, MAT_LINU>;
  constexpr int BS2 = GD * GD, MAXB = own_maxb(BS2), NAB = NN * NN, RS = R::SIZE, CCAP = FA_OWN_CCAP;
  constexpr int KMAX = (CCAP * NN + 255) / 256;
  static_assert(NAB < 127 && CCAP <= 256 && NN * GD <= 32, "contribution word / bc mask");
  __shared__ __attribute__((aligned(16))) double s_out[MAXB * BS2 + 2];
  __shared__ __attribute__((aligned(16))) double s_rec[CCAP * RS];
  __shared__ uint32_t s_mask[CCAP];
  __shared__ double s_tab[NAB * BS2];
  __shared__ uint16_t s_wd[KMAX * 256 + 256];  // lane starts, then the words [k][lane]
  __shared__ int32_t s_cell[CCAP];             // cells of the chunk after the next one
  const int tid = threadIdx.x;
  for (int t = tid; t < NAB * BS2; t += 256) s_tab[t] = P.ahat[t];
  const int64_t abase = sload(P.A.indptr, P.A.row_begin);
  const int64_t per = (P.nchunks + 7) / 8;
  // XCD-aware order (as k_gather): workgroup b walks XCD (b % 8)'s contiguous chunk range
  auto chunk_of = [&](int64_t v) -> int64_t {
    if (v >= 8 * per) return P.nchunks;
    const int64_t c = (v % 8) * per + v / 8;
    return c < P.nchunks ? c : P.nchunks;
  };
  auto nwords = [&](int64_t cc) -> int { return (int)((sload(P.cw, cc + 1) - sload(P.cw, cc)) >> 8) - 1; };
  // Prefetch registers of the next chunk: its lane program and its cells' records. They are
  // loaded at the top of a chunk and staged to LDS after that chunk's blocks are computed and
  // BEFORE its store, so waiting for them never also waits for the chunk's stores (vmcnt counts
  // stores); the compute phase reads LDS only.
  uint32_t pw[KMAX + 1];
  double pr[RS];
  uint32_t pm = 0u;
  int32_t pcell = -1, pcell2 = -1;
  auto fetch = [&](int64_t cc, int32_t cell) {
    const int K = nwords(cc);
    const uint16_t* wp = P.cwords + sload(P.cw, cc);
    pw[0] = wp[tid];
#pragma unroll
    for (int k = 0; k < KMAX; ++k) pw[k + 1] = k < K ? (uint32_t)wp[256 + k * 256 + tid] : kOwnPad;
    pcell = cell;
    if (cell >= 0) {
      const double2* rp = reinterpret_cast<const double2*>(P.rec + (int64_t)cell * RS);
#pragma unroll
      for (int q = 0; q < RS / 2; ++q) {
        const double2 t = rp[q];
        pr[2 * q] = t.x;
        pr[2 * q + 1] = t.y;
      }
      pm = P.bcmask ? P.bcmask[cell] : 0u;
    }
  };
  auto stage = [&]() {
#pragma unroll
    for (int k = 0; k <= KMAX; ++k) s_wd[k * 256 + tid] = (uint16_t)pw[k];
    if (tid < CCAP && pcell >= 0) {
      double2* dp = reinterpret_cast<double2*>(s_rec + tid * RS);
#pragma unroll
      for (int q = 0; q < RS / 2; ++q) dp[q] = make_double2(pr[2 * q], pr[2 * q + 1]);
      s_mask[tid] = pm;
    }
    if (tid < CCAP) s_cell[tid] = pcell2;
  };
  int64_t v = blockIdx.x;
  int64_t c = chunk_of(v);
  if (c >= P.nchunks) return;
  int64_t c1 = chunk_of(v + gridDim.x);
  fetch(c, tid < CCAP ? P.ccells[c * CCAP + tid] : -1);
  pcell2 = (tid < CCAP && c1 < P.nchunks) ? P.ccells[c1 * CCAP + tid] : -1;
  stage();
  __syncthreads();
  for (;;) {
    const int64_t c2 = chunk_of(v + 2 * gridDim.x);
    const int K = nwords(c);
    // the next chunk's program and records (its cells were staged last chunk), the cells of the one after
    if (c1 < P.nchunks) fetch(c1, tid < CCAP ? s_cell[tid] : -1);
    pcell2 = (tid < CCAP && c2 < P.nchunks) ? P.ccells[c2 * CCAP + tid] : -1;

    // acc sums H = sum_c sign_c (s Ji)^T B_ab (s Ji) over the block's contributions; the trace term
    // of K = H + tr(H) / (1 + lam/mu) I is linear, so it is added once per flush, not per contribution
    double acc[BS2];
#pragma unroll
    for (int e = 0; e < BS2; ++e) acc[e] = 0.0;
    const uint32_t start = s_wd[tid];
    int pos = (int)(start & 1023u);
    bool open = false;
    uint32_t lw = 0u;  // the last word summed (its cell's mask gives the block's constrained dofs)
    auto finish = [&](bool head) {
      double tr = acc[0];
#pragma unroll
      for (int i = 1; i < GD; ++i) tr += acc[i * GD + i];
      tr *= P.trc;
#pragma unroll
      for (int i = 0; i < GD; ++i) acc[i * GD + i] += tr;
      const int cs = (int)(lw & 255u), ab = (int)((lw >> 8) & 127u);
      const int a = ab / NN, b = ab - a * NN;
      const uint32_t m = s_mask[cs];
      const uint32_t lrow = (m >> (a * GD)) & ((1u << GD) - 1), lcol = (m >> (b * GD)) & ((1u << GD) - 1);
      if (lrow | lcol) {
#pragma unroll
        for (int i = 0; i < GD; ++i)
#pragma unroll
          for (int k = 0; k < GD; ++k)
            if (((lrow >> i) | (lcol >> k)) & 1u) acc[i * GD + k] = 0.0;
        if (head && a == b) {  // dolfinx set_diagonal on the constrained dofs of a diagonal block
#pragma unroll
          for (int i = 0; i < GD; ++i)
            if ((lrow >> i) & 1u) acc[i * GD + i] = P.diag;
        }
      }
    };
    if (start != kOwnIdle) {
#pragma unroll
      for (int k = 0; k < KMAX; ++k) {
        if (k < K) {  // wave-uniform
          const uint32_t w = s_wd[256 + k * 256 + tid];
          const int ab0 = (int)((w >> 8) & 127u);
          const bool valid = ab0 < NAB;  // padding: the tail of the last active lane
          const int ab = valid ? ab0 : 0;
          const int cs = valid ? (int)(w & 255u) : 0;
          double r[RS];
          {
            const double2* rp = reinterpret_cast<const double2*>(s_rec + cs * RS);
#pragma unroll
            for (int q = 0; q < RS / 2; ++q) {
              const double2 t = rp[q];
              r[2 * q] = t.x;
              r[2 * q + 1] = t.y;
            }
          }
          const double* Ah = s_tab + ab * BS2;
          double T[GD][GD];  // T = B_ab (s Ji)
#pragma unroll
          for (int i = 0; i < GD; ++i)
#pragma unroll
            for (int d = 0; d < GD; ++d) {
              double t = Ah[i * GD] * r[d];
#pragma unroll
              for (int kk = 1; kk < GD; ++kk) t = fma(Ah[i * GD + kk], r[kk * GD + d], t);
              T[i][d] = t;
            }
          const double sg = valid ? rec_sign(r[BS2]) : 0.0;  // sign of mu |J|; 0 drops a padding word
          if (__any(sg != 1.0)) {                  // rare: an inverted cell or padding in the wave
#pragma unroll
            for (int i = 0; i < GD; ++i)
#pragma unroll
              for (int d = 0; d < GD; ++d) T[i][d] *= sg;
          }
#pragma unroll
          for (int e = 0; e < GD; ++e)
#pragma unroll
            for (int d = 0; d < GD; ++d) {
              double g = acc[e * GD + d];
#pragma unroll
              for (int i = 0; i < GD; ++i) g = fma(r[i * GD + e], T[i][d], g);
              acc[e * GD + d] = g;
            }
          if (valid) {
            open = true;
            lw = w;
            if (w & 0x8000u) {  // the block's last contribution: this lane writes it (once, plain)
              finish(true);
              double* o = s_out + pos * BS2;
#pragma unroll
              for (int e = 0; e < BS2; ++e) {
                o[e] = acc[e];
                acc[e] = 0.0;
              }
              ++pos;
              open = false;
            }
          }
        }
      }
    }
    if (open) finish(false);
    __syncthreads();  // every block's plain write is done; s_rec / s_wd / s_mask are free
    if (open) {       // the segment ended inside a block: add the partial sum
      double* o = s_out + pos * BS2;
#pragma unroll
      for (int e = 0; e < BS2; ++e) atomicAdd(o + e, acc[e]);
    }
    if (c1 < P.nchunks) stage();
    __syncthreads();
    {
      const int64_t b0 = sload(P.chunk_b, c), b1 = sload(P.chunk_b, c + 1);
      const int64_t off = (b0 - abase) * BS2;
      double* out = P.A.data + off;
      const int nv = (int)(b1 - b0) * BS2;
      const int h = (int)(off & 1);
      if (h && tid == 0) __builtin_nontemporal_store(s_out[0], out);
      const int np = (nv - h) >> 1;
      typedef double dv2 __attribute__((ext_vector_type(2)));
      dv2* out2 = reinterpret_cast<dv2*>(out + h);
      constexpr int SU = kGatherStoreBatch;
      for (int t0 = tid; t0 < np; t0 += 256 * SU) {
        dv2 vv[SU];
#pragma unroll
        for (int u = 0; u < SU; ++u) {
          const int t = t0 + 256 * u;
          if (t < np) {
            if (h) { vv[u].x = s_out[1 + 2 * t]; vv[u].y = s_out[2 + 2 * t]; }
            else vv[u] = reinterpret_cast<const dv2*>(s_out)[t];
          }
        }
#pragma unroll
        for (int u = 0; u < SU; ++u) {
          const int t = t0 + 256 * u;
          if (t < np) __builtin_nontemporal_store(vv[u], out2 + t);
        }
        store_guard4(vv[0], vv[1], vv[2], vv[3]);
      }
      if (((nv - h) & 1) && tid == 0) __builtin_nontemporal_store(s_out[nv - 1], out + nv - 1);
    }
    if (c1 >= P.nchunks) break;
    __syncthreads();  // the store has read s_out
    c = c1;
    c1 = c2;
    v += gridDim.x;
  }
}

// ------------------------------------------------------------------------------------ adjacency
__global__ void k_iota(int32_t* v, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    v[i] = (int32_t)i;
}

__global__ void k_row_ptr_from_sorted(const int32_t* __restrict__ keys, int64_t n, int64_t nnodes, int64_t* __restrict__ ptr) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i <= n; i += (int64_t)gridDim.x * blockDim.x) {
    int64_t kp = (i == 0) ? -1 : keys[i - 1];
    int64_t k = (i == n) ? nnodes : keys[i];
    for (int64_t r = kp + 1; r <= k; ++r) ptr[r] = i;
  }
}

// AMD dispatches are limited to < 2^32 work-items in total (a larger grid fails silently),
// so grids are capped and every kernel is written grid-stride.
static int grid_for(int64_t n, int block = 256) {
  int64_t g = (n + block - 1) / block;
  if (g < 1) g = 1;
  if (g > kMaxBlocks) g = kMaxBlocks;
  return (int)g;
}

static int check_mesh(const fa_mesh* m) {
  if (!m || !m->cells || !m->geom || !m->x) return fail(FA_E_ARG, "mesh has null arrays");
  if (!supported(m->cell_type, m->degree)) return fail(FA_E_UNSUPPORTED, "unsupported element: cell %d degree %d", m->cell_type, m->degree);
  if (m->gdim != cell_tdim(m->cell_type)) return fail(FA_E_ARG, "gdim %d != tdim of cell %d", m->gdim, m->cell_type);
  if (m->nn != num_nodes(m->cell_type, m->degree)) return fail(FA_E_ARG, "nn %d != %d", m->nn, num_nodes(m->cell_type, m->degree));
  if (m->nv != cell_nverts(m->cell_type)) return fail(FA_E_ARG, "nv %d != %d", m->nv, cell_nverts(m->cell_type));
  if (m->ncells < 0 || m->nnodes < 0) return fail(FA_E_ARG, "negative sizes");
  if (m->ncells * (int64_t)m->nn >= (1ll << 31)) return fail(FA_E_CAPACITY, "ncells*nn = %lld exceeds int32 adjacency (shard the mesh)", (long long)(m->ncells * m->nn));
  return FA_OK;
}

extern "C" int fa_build_adjacency(const fa_mesh* mesh, int64_t* ptr, int32_t* idx, void* stream) {
  int rc = check_mesh(mesh);
  if (rc) return rc;
  if (!ptr || !idx) return fail(FA_E_ARG, "null output");
  hipStream_t s = (hipStream_t)stream;
  const int64_t n = mesh->ncells * mesh->nn;
  int end_bit = 1;
  while ((1ll << end_bit) < mesh->nnodes + 1) ++end_bit;
  int32_t *keys_out = nullptr, *vals_in = nullptr;
  void* temp = nullptr;
  size_t temp_bytes = 0;
  HIP_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, temp_bytes, mesh->cells, (int32_t*)nullptr, (int32_t*)nullptr,
                                             (int32_t*)nullptr, (int)n, 0, end_bit, s));
  HIP_TRY(hipMallocAsync((void**)&keys_out, sizeof(int32_t) * (n > 0 ? n : 1), s));
  HIP_TRY(hipMallocAsync((void**)&vals_in, sizeof(int32_t) * (n > 0 ? n : 1), s));
  HIP_TRY(hipMallocAsync(&temp, temp_bytes > 0 ? temp_bytes : 16, s));
  if (n > 0) {
    k_iota<<<grid_for(n), 256, 0, s>>>(vals_in, n);
    LAUNCH_CHECK();
    HIP_TRY(hipcub::DeviceRadixSort::SortPairs(temp, temp_bytes, mesh->cells, keys_out, vals_in, idx, (int)n, 0, end_bit, s));
  }
  k_row_ptr_from_sorted<<<grid_for(n + 1), 256, 0, s>>>(keys_out, n, mesh->nnodes, ptr);
  LAUNCH_CHECK();
  HIP_TRY(hipFreeAsync(keys_out, s));
  HIP_TRY(hipFreeAsync(vals_in, s));
  HIP_TRY(hipFreeAsync(temp, s));
  return FA_OK;
}

// ------------------------------------------------------------------------------------ sparsity
static constexpr int kSparsityCap = 2048;  // candidate (cell, node) pairs per row

// One 64-thread workgroup (one wave) per row: the nodes of the row's adjacent cells go into an LDS
// hash set (open addressing, kSparsityHash slots); its occupied slots are compacted to the row's
// distinct columns. PASS 0 counts them. PASS 1 sorts them: up to 64 in registers (a bitonic network
// over the wave's lanes, one value per lane), more in LDS (bitonic), and writes them. (Round 6: the
// candidates -- ~74 per row of config E -- were bitonic-sorted in LDS in both passes, 0.27 s.)
constexpr int kSparsityHash = 1024;  // > 2 x the distinct columns of a row the hash takes (else the LDS sort)
__device__ __forceinline__ uint32_t sp_hash(int32_t v) { return ((uint32_t)v * 0x9E3779B1u) >> (32 - 10); }
template <int PASS>
__global__ __launch_bounds__(64) void k_sparsity(MeshView M, const int64_t* __restrict__ adj_ptr,
                                                 const int32_t* __restrict__ adj_idx, int64_t* __restrict__ counts,
                                                 const int64_t* __restrict__ indptr, int32_t* __restrict__ indices,
                                                 int* err) {
  static_assert(kSparsityHash == 1024, "sp_hash: 10 bits");
  __shared__ int32_t s[kSparsityCap];
  __shared__ int32_t h[kSparsityHash];
  const int lane = threadIdx.x;
  const int nn = M.nn;
  for (int64_t r = blockIdx.x; r < M.nnodes; r += gridDim.x) {
  const int64_t j0 = adj_ptr[r], j1 = adj_ptr[r + 1];
  const int64_t ncand = (j1 - j0) * nn;
  if (ncand > kSparsityCap) {
    if (lane == 0) atomicOr(err, 4);
    continue;
  }
  __syncthreads();  // the previous row's reads of h / s are done
  auto bitonic = [&](int n2) {  // s[0, n2) ascending (n2 a power of two)
    for (int k = 2; k <= n2; k <<= 1)
      for (int j = k >> 1; j > 0; j >>= 1) {
        for (int t = lane; t < n2; t += 64) {
          const int ixj = t ^ j;
          if (ixj > t) {
            const int32_t a = s[t], b = s[ixj];
            if ((a > b) == ((t & k) == 0)) { s[t] = b; s[ixj] = a; }
          }
        }
        __syncthreads();
      }
  };
  if (ncand >= kSparsityHash / 2) {  // long rows (high-order hexahedra): sort the candidates, keep the unique
    int n2 = 1;
    while (n2 < ncand) n2 <<= 1;
    for (int t = lane; t < n2; t += 64)
      s[t] = t < ncand ? M.cells[(int64_t)(adj_idx[j0 + t / nn] / nn) * nn + t % nn] : INT32_MAX;
    __syncthreads();
    bitonic(n2);
    const int64_t base = PASS ? indptr[r] : 0;
    int running = 0;
    for (int t0 = 0; t0 < n2; t0 += 64) {
      const int t = t0 + lane;
      const int32_t v = t < n2 ? s[t] : INT32_MAX;
      const bool keep = v != INT32_MAX && (t == 0 || s[t - 1] != v);
      const unsigned long long m = __ballot(keep);
      if (PASS && keep) indices[base + running + __popcll(m & ((1ull << lane) - 1ull))] = v;
      running += __popcll(m);
    }
    if (!PASS && lane == 0) counts[r] = running;
    continue;
  }
  for (int t = lane; t < kSparsityHash; t += 64) h[t] = -1;
  __syncthreads();
  for (int t = lane; t < ncand; t += 64) {
    const int32_t v = M.cells[(int64_t)(adj_idx[j0 + t / nn] / nn) * nn + t % nn];
    uint32_t k = sp_hash(v);
    for (;;) {  // terminates: fewer than kSparsityHash / 2 values go into the table
      const int32_t prev = atomicCAS(&h[k], -1, v);
      if (prev == -1 || prev == v) break;
      k = (k + 1) & (kSparsityHash - 1);
    }
  }
  __syncthreads();
  // compaction of the occupied slots (in hash order)
  int u = 0;
  for (int t0 = 0; t0 < kSparsityHash; t0 += 64) {
    const int32_t v = h[t0 + lane];
    const bool keep = v >= 0;
    const unsigned long long m = __ballot(keep);
    if (PASS && keep) s[u + __popcll(m & ((1ull << lane) - 1ull))] = v;
    u += __popcll(m);
  }
  if (!PASS) {
    if (lane == 0) counts[r] = u;
    continue;
  }
  __syncthreads();
  const int64_t base = indptr[r];
  if (u <= 64) {  // one value per lane, bitonic across the wave (padding sorts last)
    int32_t x = lane < u ? s[lane] : INT32_MAX;
#pragma unroll
    for (int k = 2; k <= 64; k <<= 1)
#pragma unroll
      for (int j = k >> 1; j > 0; j >>= 1) {
        const int32_t y = __shfl_xor(x, j);
        const bool up = (lane & k) == 0, lo = (lane & j) == 0;
        x = (lo == up) ? min(x, y) : max(x, y);
      }
    if (lane < u) indices[base + lane] = x;
  } else if (u <= 128) {  // two per lane (elements lane and lane + 64; config E's vertex rows hold ~65)
    int32_t x0 = s[lane], x1 = 64 + lane < u ? s[64 + lane] : INT32_MAX;
#pragma unroll
    for (int k = 2; k <= 128; k <<= 1)
#pragma unroll
      for (int j = k >> 1; j > 0; j >>= 1) {
        if (j == 64) {  // partners in one lane (k = 128: ascending)
          const int32_t a = min(x0, x1), b = max(x0, x1);
          x0 = a;
          x1 = b;
        } else {
          const bool lo = (lane & j) == 0;
          const bool up0 = (lane & k) == 0, up1 = ((64 + lane) & k) == 0;
          const int32_t y0 = __shfl_xor(x0, j), y1 = __shfl_xor(x1, j);
          x0 = (lo == up0) ? min(x0, y0) : max(x0, y0);
          x1 = (lo == up1) ? min(x1, y1) : max(x1, y1);
        }
      }
    indices[base + lane] = x0;  // u > 64
    if (64 + lane < u) indices[base + 64 + lane] = x1;
  } else {
    int n2 = 1;
    while (n2 < u) n2 <<= 1;
    for (int t = u + lane; t < n2; t += 64) s[t] = INT32_MAX;
    __syncthreads();
    bitonic(n2);
    for (int t = lane; t < u; t += 64) indices[base + t] = s[t];
  }
  }
}

extern "C" int fa_sparsity_count(const fa_mesh* mesh, const fa_adjacency* adj, int64_t* indptr, int64_t* nblocks,
                                 void* stream) {
  int rc = check_mesh(mesh);
  if (rc) return rc;
  if (!adj || !adj->ptr || !adj->idx || !indptr) return fail(FA_E_ARG, "null argument");
  hipStream_t s = (hipStream_t)stream;
  MeshView M{mesh->cells, mesh->geom, mesh->x, mesh->ncells, mesh->nnodes, mesh->nn, mesh->nv, mesh->gdim};
  int* derr = nullptr;
  int64_t* counts = nullptr;
  void* temp = nullptr;
  size_t temp_bytes = 0;
  const int64_t n = mesh->nnodes;
  HIP_TRY(hipMallocAsync((void**)&derr, sizeof(int), s));
  HIP_TRY(hipMemsetAsync(derr, 0, sizeof(int), s));
  HIP_TRY(hipMallocAsync((void**)&counts, sizeof(int64_t) * (n + 1), s));
  HIP_TRY(hipMemsetAsync(counts, 0, sizeof(int64_t) * (n + 1), s));
  if (n > 0) {
    k_sparsity<0><<<grid_for(n, 1), 64, 0, s>>>(M, adj->ptr, adj->idx, counts, nullptr, nullptr, derr);
    LAUNCH_CHECK();
  }
  HIP_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, temp_bytes, counts, indptr, (int)(n + 1), s));
  HIP_TRY(hipMallocAsync(&temp, temp_bytes > 0 ? temp_bytes : 16, s));
  HIP_TRY(hipcub::DeviceScan::ExclusiveSum(temp, temp_bytes, counts, indptr, (int)(n + 1), s));
  int herr = 0;
  HIP_TRY(hipMemcpyAsync(&herr, derr, sizeof(int), hipMemcpyDeviceToHost, s));
  HIP_TRY(hipMemcpyAsync(nblocks, indptr + n, sizeof(int64_t), hipMemcpyDeviceToHost, s));
  HIP_TRY(hipFreeAsync(temp, s));
  HIP_TRY(hipFreeAsync(counts, s));
  HIP_TRY(hipFreeAsync(derr, s));
  HIP_TRY(hipStreamSynchronize(s));
  if (herr) return fail(FA_E_CAPACITY, "a row has more than %d (cell, node) candidates", kSparsityCap);
  return FA_OK;
}

extern "C" int fa_sparsity_fill(const fa_mesh* mesh, const fa_adjacency* adj, const int64_t* indptr, int32_t* indices,
                                void* stream) {
  int rc = check_mesh(mesh);
  if (rc) return rc;
  if (!adj || !adj->ptr || !adj->idx || !indptr || !indices) return fail(FA_E_ARG, "null argument");
  hipStream_t s = (hipStream_t)stream;
  MeshView M{mesh->cells, mesh->geom, mesh->x, mesh->ncells, mesh->nnodes, mesh->nn, mesh->nv, mesh->gdim};
  int* derr = nullptr;
  HIP_TRY(hipMallocAsync((void**)&derr, sizeof(int), s));
  HIP_TRY(hipMemsetAsync(derr, 0, sizeof(int), s));
  if (mesh->nnodes > 0) {
    k_sparsity<1><<<grid_for(mesh->nnodes, 1), 64, 0, s>>>(M, adj->ptr, adj->idx, nullptr, indptr, indices, derr);
    LAUNCH_CHECK();
  }
  int herr = 0;
  HIP_TRY(hipMemcpyAsync(&herr, derr, sizeof(int), hipMemcpyDeviceToHost, s));
  HIP_TRY(hipFreeAsync(derr, s));
  HIP_TRY(hipStreamSynchronize(s));
  if (herr) return fail(FA_E_CAPACITY, "a row has more than %d (cell, node) candidates", kSparsityCap);
  return FA_OK;
}

// ------------------------------------------------------------------------------------ gather plan
// slot map: thread per row node; for each adjacency entry of the row and each column node of the
// cell, the position of that column in the row (binary search once, at plan time)
// ------------------------------------------------------------------------------ pattern check
static int scratch_alloc(void** p, size_t bytes, hipStream_t s);
// fa_check_pattern: the sparsity pattern and the node -> cell adjacency are built with rocPRIM sorts
// and scans (whose gfx950 code the library does not control, tools/store_hazard.py); this validates
// both on the device. One thread per row: indptr monotone, columns in range and strictly increasing;
// adjacency entries of row r sorted, unique and at a dofmap position holding node r; every node of
// every adjacent cell found in the row (its block marked in `hit`); then every block marked (no
// column that no cell needs). Error bits: 1 indptr, 2 columns, 4 missing pair, 8 extra column,
// 32 adjacency.
__global__ void k_check_pattern(MeshView M, const int64_t* __restrict__ adj_ptr, const int32_t* __restrict__ adj_idx,
                                const int64_t* __restrict__ indptr, const int32_t* __restrict__ indices,
                                int64_t nblocks, uint8_t* __restrict__ hit, int* err) {
  const int nn = M.nn;
  const int64_t nent = M.ncells * nn;
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < M.nnodes; r += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b0 = indptr[r], b1 = indptr[r + 1];
    if (b1 < b0 || b0 < 0 || b1 > nblocks) {
      atomicOr(err, 1);
      continue;
    }
    int e = 0;
    for (int64_t k = b0; k < b1; ++k) {
      const int32_t c = indices[k];
      if (c < 0 || c >= M.nnodes || (k > b0 && indices[k - 1] >= c)) e |= 2;
    }
    const int64_t j0 = adj_ptr[r], j1 = adj_ptr[r + 1];
    if (j1 < j0 || j0 < 0 || j1 > nent) e |= 32;
    for (int64_t j = j0; j < j1 && !(e & 32); ++j) {
      const int32_t p = adj_idx[j];
      if (p < 0 || p >= nent || M.cells[p] != r || (j > j0 && adj_idx[j - 1] >= p)) {
        e |= 32;
        break;
      }
      const int64_t c = p / nn;
      for (int b = 0; b < nn; ++b) {
        const int32_t col = M.cells[c * nn + b];
        int64_t lo = b0, hi = b1 - 1, f = -1;
        while (lo <= hi) {
          const int64_t mid = (lo + hi) >> 1;
          const int32_t v = indices[mid];
          if (v == col) { f = mid; break; }
          if (v < col) lo = mid + 1; else hi = mid - 1;
        }
        if (f < 0) e |= 4;
        else hit[f] = 1;
      }
    }
    if (e) atomicOr(err, e);
  }
}
__global__ void k_check_hits(const uint8_t* __restrict__ hit, int64_t n, int* err) {
  int e = 0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    if (!hit[i]) e = 8;
  if (e) atomicOr(err, e);
}

// exact: also refuse a block no cell needs (bit 8: the pattern create_matrix builds). Assembling into
// a superset pattern is valid (dolfinx / PETSc accept one: a rank's slab pattern, a pattern with room
// for later entries), so fa_assemble_matrix's FA_CHECK_ERRORS checks without it.
static int check_pattern(const fa_mesh* mesh, const fa_adjacency* adj, const int64_t* indptr,
                         const int32_t* indices, int64_t nblocks, bool exact, void* stream) {
  int rc = check_mesh(mesh);
  if (rc) return rc;
  if (!adj || !adj->ptr || !adj->idx || !indptr || (!indices && nblocks > 0)) return fail(FA_E_ARG, "null argument");
  if (nblocks < 0) return fail(FA_E_ARG, "negative block count");
  hipStream_t s = (hipStream_t)stream;
  const int64_t n = mesh->nnodes;
  int64_t h[4] = {0, 0, 0, 0};
  HIP_TRY(hipMemcpyAsync(&h[0], indptr, sizeof(int64_t), hipMemcpyDeviceToHost, s));
  HIP_TRY(hipMemcpyAsync(&h[1], indptr + n, sizeof(int64_t), hipMemcpyDeviceToHost, s));
  HIP_TRY(hipMemcpyAsync(&h[2], adj->ptr, sizeof(int64_t), hipMemcpyDeviceToHost, s));
  HIP_TRY(hipMemcpyAsync(&h[3], adj->ptr + n, sizeof(int64_t), hipMemcpyDeviceToHost, s));
  MeshView M{mesh->cells, mesh->geom, mesh->x, mesh->ncells, mesh->nnodes, mesh->nn, mesh->nv, mesh->gdim};
  int* derr = nullptr;
  uint8_t* hit = nullptr;
  HIP_TRY(hipMallocAsync((void**)&derr, sizeof(int), s));
  HIP_TRY(hipMemsetAsync(derr, 0, sizeof(int), s));
  if ((rc = scratch_alloc((void**)&hit, (size_t)std::max<int64_t>(nblocks, 1), s))) return rc;
  HIP_TRY(hipMemsetAsync(hit, 0, (size_t)std::max<int64_t>(nblocks, 1), s));
  if (n > 0) {
    k_check_pattern<<<grid_for(n), 256, 0, s>>>(M, adj->ptr, adj->idx, indptr, indices, nblocks, hit, derr);
    LAUNCH_CHECK();
  }
  if (nblocks > 0 && exact) {
    k_check_hits<<<grid_for(nblocks), 256, 0, s>>>(hit, nblocks, derr);
    LAUNCH_CHECK();
  }
  int herr = 0;
  HIP_TRY(hipMemcpyAsync(&herr, derr, sizeof(int), hipMemcpyDeviceToHost, s));
  HIP_TRY(hipFreeAsync(hit, s));
  HIP_TRY(hipFreeAsync(derr, s));
  HIP_TRY(hipStreamSynchronize(s));
  if (h[0] != 0 || h[1] != nblocks)
    return fail(FA_E_PATTERN, "pattern: indptr[0] = %lld, indptr[nnodes] = %lld for %lld blocks", (long long)h[0],
                (long long)h[1], (long long)nblocks);
  if (h[2] != 0 || h[3] != mesh->ncells * mesh->nn)
    return fail(FA_E_PATTERN, "adjacency: ptr[0] = %lld, ptr[nnodes] = %lld for %lld entries", (long long)h[2],
                (long long)h[3], (long long)(mesh->ncells * mesh->nn));
  if (herr)
    return fail(FA_E_PATTERN, "pattern check failed (bits %d:%s%s%s%s%s)", herr, (herr & 1) ? " indptr" : "",
                (herr & 2) ? " columns out of range or unsorted" : "", (herr & 4) ? " a cell's (row, column) pair missing" : "",
                (herr & 8) ? " a column no cell needs" : "", (herr & 32) ? " adjacency" : "");
  return FA_OK;
}

extern "C" int fa_check_pattern(const fa_mesh* mesh, const fa_adjacency* adj, const int64_t* indptr,
                                const int32_t* indices, int64_t nblocks, void* stream) {
  return check_pattern(mesh, adj, indptr, indices, nblocks, true, stream);
}

// One wave per row (round 6; a thread per row took 0.21 s on config E): the row's columns are
// staged in LDS (rows of up to kSlotCols blocks; longer rows search the pattern in memory) and the
// lanes take the row's (adjacency entry, column node) pairs in order, so the slot writes of a row are
// one contiguous run of u16.
constexpr int kSlotCols = 1024;
__global__ __launch_bounds__(64) void k_build_slots(MeshView M, const int64_t* __restrict__ adj_ptr,
                                                    const int32_t* __restrict__ adj_idx,
                                                    const int64_t* __restrict__ indptr,
                                                    const int32_t* __restrict__ indices, uint16_t* __restrict__ slots,
                                                    int* err) {
  __shared__ int32_t cols[kSlotCols];
  const int nn = M.nn;
  const int lane = threadIdx.x;
  for (int64_t r = blockIdx.x; r < M.nnodes; r += gridDim.x) {
    const int64_t b0 = indptr[r], b1 = indptr[r + 1];
    const int64_t nb = b1 - b0;
    if (nb > 65535) {
      if (lane == 0) atomicOr(err, 8);
      continue;
    }
    const bool inl = nb <= kSlotCols;
    __syncthreads();  // the previous row's searches are done
    if (inl)
      for (int t = lane; t < nb; t += 64) cols[t] = indices[b0 + t];
    __syncthreads();
    const int64_t j0 = adj_ptr[r], nc = (adj_ptr[r + 1] - j0) * nn;
    for (int64_t t = lane; t < nc; t += 64) {
      const int64_t j = j0 + t / nn;
      const int b = (int)(t % nn);
      const int32_t col = M.cells[(int64_t)(adj_idx[j] / nn) * nn + b];
      int64_t lo = 0, hi = nb - 1, s = -1;
      while (lo <= hi) {
        const int64_t mid = (lo + hi) >> 1;
        const int32_t v = inl ? cols[mid] : indices[b0 + mid];
        if (v == col) { s = mid; break; }
        if (v < col) lo = mid + 1; else hi = mid - 1;
      }
      if (s < 0) { atomicOr(err, 1); s = 0; }
      slots[j * nn + b] = (uint16_t)s;
    }
  }
}

extern "C" int fa_plan_slots(const fa_mesh* mesh, const fa_adjacency* adj, const fa_bsr* A, uint16_t* slots,
                             fa_plan* plan, void* stream) {
  int rc = check_mesh(mesh);
  if (rc) return rc;
  if (!adj || !A || !slots || !plan) return fail(FA_E_ARG, "null argument");
  hipStream_t s = (hipStream_t)stream;
  MeshView M{mesh->cells, mesh->geom, mesh->x, mesh->ncells, mesh->nnodes, mesh->nn, mesh->nv, mesh->gdim};
  int* derr = nullptr;
  HIP_TRY(hipMallocAsync((void**)&derr, sizeof(int), s));
  HIP_TRY(hipMemsetAsync(derr, 0, sizeof(int), s));
  if (mesh->nnodes > 0) {
    k_build_slots<<<grid_for(mesh->nnodes, 1), 64, 0, s>>>(M, adj->ptr, adj->idx, A->indptr, A->indices, slots, derr);
    LAUNCH_CHECK();
  }
  int herr = 0;
  HIP_TRY(hipMemcpyAsync(&herr, derr, sizeof(int), hipMemcpyDeviceToHost, s));
  HIP_TRY(hipFreeAsync(derr, s));
  HIP_TRY(hipStreamSynchronize(s));
  if (herr & 8) return fail(FA_E_CAPACITY, "a row holds more than 65535 blocks");
  if (herr) return fail(FA_E_PATTERN, "sparsity pattern misses a (row, column) pair of a cell");
  plan->slots = slots;
  plan->slot_order = 0;
  plan->eadj = nullptr;
  return FA_OK;
}

// Bank-conflict-aware item order (fa_plan_order). An item's NBG blocks are added one per step of
// its rolled block loop, 9 ds_add_f64 each, all lanes of a wave at the same step. Measured LDS
// model (tools/probe/lds_bank_probe.hip, gfx950): a 64-bit LDS op serves each 16-lane quarter of
// the wave on its own, and two lanes of a quarter conflict when their slots are equal mod 16
// (72-B blocks); k lanes on one residue cost k passes, lanes on one slot a little more. Within each
// quarter of the kernel's item -> lane mapping the order in which every lane visits its NBG column
// slots is chosen to minimise sum over steps of the largest residue count (the passes), with the
// sum of squared counts as tie-break: identity start, then pairwise step swaps per lane until no
// swap improves. The slot map then holds (b << 10) | position in that order. One thread per
// (chunk, quarter).
// Positional plans (eperm != NULL): position jj of a chunk holds entry eperm[a0 + jj]; the plain
// map is read from src and written by position, with chunk-relative block positions.
// alternating-path moves of the slot order search (k_order_slots): rounds (with FA_PLAN_ORDER_SEARCH)
// and lanes per chain. Opt-in since round 5: on config E they took the plan from 1.7 to 20 s for
// 37.6 -> 37.4 ms per assembly (break-even after ~90,000 assemblies; the reference assembles J a few
// times per Newton solve)
constexpr int kKempeRounds = 4;
constexpr int kKempeLen = 6;
// The search's per-thread state (residues, picks, counts, step maxima) sits in LDS, one slice per
// thread of a 64-thread workgroup (round 5; in scratch it made the search with the alternating-path
// moves a 19.6-s launch on config E).
constexpr int kOrderThreads = 64;
template <int NN, int NSPLIT>
__global__ __launch_bounds__(kOrderThreads) void k_order_slots(const int64_t* __restrict__ row_start,
                                                                const int64_t* __restrict__ indptr,
                                                                const int64_t* __restrict__ adj_ptr, int64_t nchunks,
                                                                int groups_per_chunk, uint16_t* __restrict__ slots,
                                                                const uint16_t* __restrict__ src,
                                                                const uint16_t* __restrict__ eperm, int rounds) {
  constexpr int NBG = NN / NSPLIT, Q = 16;
  __shared__ uint8_t s_res[kOrderThreads][Q][NBG], s_pick[kOrderThreads][Q][NBG], s_cnt[kOrderThreads][NBG][16];
  __shared__ int s_mx[kOrderThreads][NBG], s_nmx[kOrderThreads][NBG];
  auto& res = s_res[threadIdx.x];
  auto& pick = s_pick[threadIdx.x];
  auto& cnt = s_cnt[threadIdx.x];
  auto& mx = s_mx[threadIdx.x];
  auto& nmx = s_nmx[threadIdx.x];
  const int64_t total = nchunks * groups_per_chunk;
  for (int64_t gid = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; gid < total;
       gid += (int64_t)gridDim.x * blockDim.x) {
    const int64_t c = gid / groups_per_chunk;
    const int g = (int)(gid % groups_per_chunk);
    const int64_t r0 = row_start[c], r1 = row_start[c + 1];
    const int64_t a0 = adj_ptr[r0];
    const int na = (int)(adj_ptr[r1] - a0);
    const int nitems = na * NSPLIT;
    const int p0 = Q * g;
    if (p0 >= nitems) continue;
    const int64_t b0 = indptr[r0];
    const int st = gather_perm_stride(na);
    const float inv = 1.0f / (float)na;
    const int nl = min(Q, nitems - p0);
    uint16_t off[Q][NBG];
    int64_t ent[Q];
    int base[Q];
    const uint16_t* rd = eperm ? src : slots;
    for (int t = 0; t < NBG; ++t)
      for (int r = 0; r < 16; ++r) cnt[t][r] = 0;
    for (int q = 0; q < nl; ++q) {
      const int p = p0 + q;
      const int part = p % NSPLIT;
      const int j = eperm ? (int)eperm[a0 + p / NSPLIT] : gather_perm(p / NSPLIT, na, st, inv);
      const int64_t e = a0 + j;
      int64_t lo = r0, hi = r1 - 1;  // row of entry e: adj_ptr[row] <= e < adj_ptr[row + 1]
      while (lo < hi) {
        const int64_t mid = (lo + hi + 1) >> 1;
        if (adj_ptr[mid] <= e) lo = mid; else hi = mid - 1;
      }
      const int rowlo = (int)(indptr[lo] - b0);
      base[q] = eperm ? rowlo : 0;
      const int64_t ein = e * NN + part * NBG;
      ent[q] = (eperm ? a0 + p / NSPLIT : e) * NN + part * NBG;
      for (int t = 0; t < NBG; ++t) {
        off[q][t] = rd[ein + t];
        res[q][t] = (uint8_t)((rowlo + off[q][t]) & 15);
        pick[q][t] = (uint8_t)t;
        ++cnt[t][res[q][t]];
      }
    }
    // step maxima and how many residues reach them: a swap is then priced in O(1) and the two
    // steps are recounted only when it is taken
    auto recount = [&](int t) {
      int m = 0, n = 0;
      for (int r = 0; r < 16; ++r) {
        const int v = cnt[t][r];
        if (v > m) { m = v; n = 1; } else if (v == m) ++n;
      }
      mx[t] = m;
      nmx[t] = n;
    };
    // new maximum of step t after one add moves from residue ro (count co) to rn (count cn)
    auto moved_max = [&](int t, int co, int cn) {
      if (cn + 1 > mx[t]) return cn + 1;
      if (co == mx[t] && nmx[t] == 1 && cn + 1 < mx[t]) return mx[t] - 1;
      return mx[t];
    };
    for (int t = 0; t < NBG; ++t) recount(t);
    auto swap_pick = [&](int q, int t1, int t2) {
      const int ra = res[q][pick[q][t1]], rb = res[q][pick[q][t2]];
      --cnt[t1][ra]; ++cnt[t1][rb]; --cnt[t2][rb]; ++cnt[t2][ra];
      const uint8_t x = pick[q][t1];
      pick[q][t1] = pick[q][t2];
      pick[q][t2] = x;
      recount(t1);
      recount(t2);
    };
    auto descend = [&]() {
      for (int pass = 0; pass < 32; ++pass) {
        bool improved = false;
        for (int q = 0; q < nl; ++q)
          for (int t1 = 0; t1 < NBG; ++t1)
            for (int t2 = t1 + 1; t2 < NBG; ++t2) {
              const int ra = res[q][pick[q][t1]], rb = res[q][pick[q][t2]];
              if (ra == rb) continue;
              const int a1 = cnt[t1][ra], b1 = cnt[t1][rb], a2 = cnt[t2][ra], b2 = cnt[t2][rb];
              // step t1: ra -> rb; step t2: rb -> ra
              const int d = moved_max(t1, a1, b1) + moved_max(t2, b2, a2) - mx[t1] - mx[t2];
              const int sq = 2 * (b1 - a1) + 2 + 2 * (a2 - b2) + 2;
              if (d < 0 || (d == 0 && sq < 0)) {
                swap_pick(q, t1, t2);
                improved = true;
              }
            }
        if (!improved) break;
      }
    };
    descend();
    // Alternating-path (Kempe) moves between two steps, which the pairwise descent cannot make: a
    // lane on a residue that two lanes hit at step t1 swaps its blocks of steps t1 and t2; the
    // residue it brings to t1 may collide there with another lane, which swaps its t1 / t2 blocks
    // too, and so on (at most kKempeLen lanes). A chain is kept when the two steps' passes drop,
    // otherwise undone; then the descent runs again. (config E: passes 1.30 x the per-quarter bound
    // max(steps, largest residue count) after the descent alone; tools/r4/plan_stats.py)
    if constexpr (NBG > 1) {
      auto res_at = [&](int q, int t) { return (int)res[q][pick[q][t]]; };
      for (int round = 0; round < rounds; ++round) {
        bool improved = false;
        for (int t1 = 0; t1 < NBG; ++t1) {
          for (int r = 0; r < 16; ++r) {
            if (cnt[t1][r] < 2) continue;
            int q0 = -1;
            for (int q = 0; q < nl; ++q)
              if (res_at(q, t1) == r) { q0 = q; break; }
            bool done = false;
            for (int t2 = 0; t2 < NBG && !done; ++t2) {
              if (t2 == t1) continue;
              const int before = mx[t1] + mx[t2];
              int path[kKempeLen], len = 0;
              int q = q0;
              while (true) {
                swap_pick(q, t1, t2);
                path[len++] = q;
                const int rn = res_at(q, t1);  // brought from t2
                if (cnt[t1][rn] < 2 || len == kKempeLen) break;
                int qn = -1;
                for (int qq = 0; qq < nl && qn < 0; ++qq) {
                  if (res_at(qq, t1) != rn) continue;
                  bool used = false;
                  for (int l = 0; l < len; ++l) used |= path[l] == qq;
                  if (!used) qn = qq;
                }
                if (qn < 0) break;
                q = qn;
              }
              if (mx[t1] + mx[t2] < before) {
                done = improved = true;
              } else {
                for (int l = len - 1; l >= 0; --l) swap_pick(path[l], t1, t2);
              }
            }
            if (done) break;  // counts changed: rescan from the next step
          }
        }
        if (!improved) break;
        descend();
      }
    }
    for (int q = 0; q < nl; ++q) {
      const int part = (p0 + q) % NSPLIT;
      uint16_t v[NBG];
      for (int t = 0; t < NBG; ++t) {
        const int k = pick[q][t];
        v[t] = (uint16_t)(((part * NBG + k) << 10) | (base[q] + off[q][k]));
      }
      // one 2-B store each (volatile: not merged into 12- / 16-B stores, whose data registers the
      // compiler reuses within the gfx950 store-data hazard window; tests/test_store_hazard.py)
      volatile uint16_t* so = slots + ent[q];
      for (int t = 0; t < NBG; ++t) so[t] = v[t];
    }
  }
}

// Positional plan, step 1 (fa_plan_order with an entry buffer): which adjacency entries of a
// chunk share a 16-lane quarter. Entries are placed one by one (in the kernel's default entry
// permutation, which spreads rows) into the quarter with room whose residue histogram (slots
// mod 16 over all its lanes' blocks) overlaps the entry's residues least, so that no residue
// collects many more adds than the quarter has steps; the order search then spreads them over
// the steps. Writes eperm (position -> entry offset) and eadj (the entries' adjacency values in
// position order). One thread per chunk.
// The residue histograms and fill counts of a chunk's quarters live in LDS (round 6: a thread's 1 KB
// array of up to 64 quarters sat in scratch; config E's plan step 0.10 s), sized by MQ quarters: the
// host picks MQ = 16 when every chunk holds at most 16 quarters (the k_gather_lin / k_gather_neo
// plans: <= 256 items per chunk), else kGatherMaxAdj / EQ.
constexpr int kPermThreads = 64;
template <int NN, int NSPLIT, int MQ>
__global__ __launch_bounds__(kPermThreads) void k_plan_perm(const int64_t* __restrict__ row_start,
                                                            const int64_t* __restrict__ indptr,
                                                            const int64_t* __restrict__ adj_ptr,
                                                            const int32_t* __restrict__ adj_idx, int64_t nchunks,
                                                            const uint16_t* __restrict__ src,
                                                            uint16_t* __restrict__ eperm, int32_t* __restrict__ eadj) {
  constexpr int EQ = NSPLIT <= 16 ? 16 / NSPLIT : 1;  // entries per quarter (host: only for 16 % NSPLIT == 0)
  constexpr int TH = MQ <= 16 ? kPermThreads : 16;  // threads per workgroup (the host launches TH)
  __shared__ uint8_t s_h[TH][MQ][16], s_fill[TH][MQ];
  auto& h = s_h[threadIdx.x];
  auto& fill = s_fill[threadIdx.x];
  for (int64_t c = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; c < nchunks;
       c += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r0 = row_start[c], r1 = row_start[c + 1];
    const int64_t a0 = adj_ptr[r0];
    const int na = (int)(adj_ptr[r1] - a0);
    if (na <= 0) continue;
    const int64_t b0 = indptr[r0];
    const int nq = min((na + EQ - 1) / EQ, MQ);
    for (int q = 0; q < nq; ++q) {
      fill[q] = 0;
      for (int r = 0; r < 16; ++r) h[q][r] = 0;
    }
    const int st = gather_perm_stride(na);
    const float inv = 1.0f / (float)na;
    for (int jj = 0; jj < na; ++jj) {
      const int j = gather_perm(jj, na, st, inv);
      const int64_t e = a0 + j;
      int64_t lo = r0, hi = r1 - 1;
      while (lo < hi) {
        const int64_t mid = (lo + hi + 1) >> 1;
        if (adj_ptr[mid] <= e) lo = mid; else hi = mid - 1;
      }
      const int rowlo = (int)(indptr[lo] - b0);
      uint8_t res[NN];
      for (int b = 0; b < NN; ++b) res[b] = (uint8_t)((rowlo + src[e * NN + b]) & 15);
      int best = -1, bc = 1 << 30;
      for (int q = 0; q < nq; ++q) {
        const int cap = q + 1 < nq ? EQ : na - EQ * (nq - 1);
        if (fill[q] >= cap) continue;
        int cost = 0;
        for (int b = 0; b < NN; ++b) cost += h[q][res[b]];
        if (cost < bc) { bc = cost; best = q; }
      }
      const int pos = best * EQ + fill[best];
      ++fill[best];
      for (int b = 0; b < NN; ++b) ++h[best][res[b]];
      eperm[a0 + pos] = (uint16_t)j;
      eadj[a0 + pos] = adj_idx[e];
    }
  }
}

// NSPLIT of the affine-simplex linear-elasticity gather kernel for (cell, degree, quadrature
// points), or 0 when that kernel does not exist (must match dispatch_gather)
constexpr int FA_P2TET_NSPLIT = 2;  // measured best with the reference-tensor blocks (n=120 sweep)
// affine tensor cells: column nodes per item = NN / NSPLIT
constexpr int FA_Q2HEX_NSPLIT = 9;
constexpr int FA_Q3HEX_NSPLIT = 32;
// Q2 quadrilaterals: whole entries (9 blocks per item) since round 6, when affine ones moved to
// k_gather_lin: its positional plans fill 16-lane quarters with whole entries (16 % NSPLIT == 0), which
// 3 does not divide (the generic gather had used 3 with searched slots)
constexpr int FA_Q2QUAD_NSPLIT = 1;
constexpr int FA_P1TET_NSPLIT = 1;  // P1 tetrahedra: whole entries (4 blocks per item); config C 1.86 vs 1.97 ms (2), 2.25 (4)
// k_gather_lin's workgroup size (one item per thread, chunks of up to NT / NSPLIT entries): P1
// tetrahedra have 4-block items, so their chunks are short on work per barrier at 256 items
constexpr int FA_P1TET_NT = 256;  // 512 measured 1.72 vs 1.68 ms on config C
constexpr int FA_P2TET_NT = 256;
// affine Q2 quadrilaterals (whole 9-block entries): the 1023-block cap of a chunk binds at ~144
// entries, so 256-item workgroups ran half empty; 128 items measured config B 0.534 vs 0.612 ms
// (192: 0.572; 128 items with a 767 / 511-block accumulator for more resident workgroups: 0.574 /
// 0.640; 64 items: 0.59-0.66; profiles/r6/q2quad_nt_ab.txt)
constexpr int FA_Q2QUAD_NT = 128;
__host__ __device__ constexpr int lin_threads(int gd, int nn) {
  return gd == 3 && nn == 4 ? FA_P1TET_NT : gd == 3 && nn == 10 ? FA_P2TET_NT : gd == 2 && nn == 9 ? FA_Q2QUAD_NT : 256;
}
static int lin_simplex_nsplit(int ct, int p, int nq, bool affine = false) {
  // affine hexahedra (MAT_AFFT): Q1 / Q2 / Q3 with their default rules
  if (affine && ct == FA_HEXAHEDRON && p == 1 && nq == 8) return 2;
  if (affine && ct == FA_HEXAHEDRON && p == 2 && nq == 27) return FA_Q2HEX_NSPLIT;
  if (affine && ct == FA_HEXAHEDRON && p == 3 && nq == 64) return FA_Q3HEX_NSPLIT;
  if (affine && ct == FA_QUADRILATERAL && p == 1 && nq == 4) return 1;
  if (affine && ct == FA_QUADRILATERAL && p == 2 && nq == 9) return FA_Q2QUAD_NSPLIT;
  if (affine && ct == FA_QUADRILATERAL && p == 3 && nq == 16) return 4;
  if (ct == FA_TRIANGLE && p == 1 && nq == 1) return 1;
  if (ct == FA_TRIANGLE && p == 2 && nq == 3) return 2;
  if (ct == FA_TETRAHEDRON && p == 1 && nq == 1) return FA_P1TET_NSPLIT;
  if (ct == FA_TETRAHEDRON && p == 2 && nq == 4) return FA_P2TET_NSPLIT;
  return 0;
}

extern "C" int fa_plan_order(const fa_mesh* mesh, const fa_adjacency* adj, const fa_bsr* A, int32_t* eadj,
                             fa_plan* plan, void* stream) {
  int rc = check_mesh(mesh);
  if (rc) return rc;
  if (!adj || !A || !plan) return fail(FA_E_ARG, "null argument");
  if (!plan->slots) return fail(FA_E_ARG, "fa_plan_order needs the slot map (fa_plan_slots first)");
  plan->slot_order = 0;
  plan->eadj = nullptr;
  DevTables T;
  if ((rc = get_tables(mesh->cell_type, mesh->degree, -1, &T))) return rc;
  const int ns = (plan->cell_flags & FA_PLAN_NEO) && is_simplex(mesh->cell_type)
                     ? neo_nsplit(mesh->cell_type, mesh->degree)
                     : lin_simplex_nsplit(mesh->cell_type, mesh->degree, T.nq, (plan->cell_flags & FA_PLAN_AFFINE) != 0);
  if (ns == 0 || plan->nchunks <= 0) return FA_OK;  // no kernel reads an ordered map: keep plain slots
  // ordered entries pack (b << 10) | chunk-relative position (k_order_slots): keep the plain map
  // for a plan whose chunks could hold 1024 blocks or more
  if (plan->max_blocks >= 1024 || gather_maxb(false, mesh->gdim * mesh->gdim) >= 1024) return FA_OK;
  // 16-lane quarters per chunk: the plan's largest chunk decides (round 6; every chunk had been given
  // kGatherMaxAdj * ns / 16 threads, most of which found no items)
  const int groups = (int)((std::min<int64_t>(std::max<int32_t>(plan->max_adj, 1), kGatherMaxAdj) * ns + 15) / 16);
  const int rounds = (plan->cell_flags & FA_PLAN_ORDER_SEARCH) ? kKempeRounds : 0;
  hipStream_t s = (hipStream_t)stream;
  const int64_t total = plan->nchunks * groups;
  uint16_t* sl = const_cast<uint16_t*>(plan->slots);
  // positional plan: the plain map is copied aside (the order kernel rewrites by position). Only
  // for the kernels that read one (k_gather's POSM: an entry's items fill whole 16-lane quarters,
  // and affine tensor cells only with a full bc mask, NN * GD <= 32)
  const bool tensor = mesh->cell_type == FA_HEXAHEDRON || mesh->cell_type == FA_QUADRILATERAL;
  const bool posn = eadj != nullptr && 16 % ns == 0 && !(tensor && mesh->nn * mesh->gdim > 32);
  uint16_t *src = nullptr, *eperm = nullptr;
  const int64_t nent = mesh->ncells * mesh->nn;
  // k_plan_perm's quarter arrays: 16 quarters cover every chunk of <= 16 x 16 items
  const bool small_q = (int64_t)std::max<int32_t>(plan->max_adj, 1) * ns <= 256;
  if (posn) {
    HIP_TRY(hipMallocAsync((void**)&src, sizeof(uint16_t) * nent * mesh->nn, s));
    HIP_TRY(hipMallocAsync((void**)&eperm, sizeof(uint16_t) * nent, s));
    HIP_TRY(hipMemcpyAsync(src, sl, sizeof(uint16_t) * nent * mesh->nn, hipMemcpyDeviceToDevice, s));
  }
#define ORD(NN_, NS_)                                                                                         \
  do {                                                                                                        \
    if (posn && small_q)                                                                                      \
      k_plan_perm<NN_, NS_, 16><<<grid_for(plan->nchunks, kPermThreads), kPermThreads, 0, s>>>(               \
          plan->row_start, A->indptr, adj->ptr, adj->idx, plan->nchunks, src, eperm, eadj);                      \
    else if (posn)                                                                                            \
      k_plan_perm<NN_, NS_, kGatherMaxAdj / (NS_ <= 16 ? 16 / NS_ : 1)><<<grid_for(plan->nchunks, 16), 16, 0, s>>>( \
          plan->row_start, A->indptr, adj->ptr, adj->idx, plan->nchunks, src, eperm, eadj);                      \
    k_order_slots<NN_, NS_><<<grid_for(total, kOrderThreads), kOrderThreads, 0, s>>>(plan->row_start, A->indptr, adj->ptr, plan->nchunks, \
                                                            groups, sl, src, eperm, rounds);                   \
  } while (0)
  bool ok = true;
  if (mesh->nn == 3 && ns == 1) ORD(3, 1);
  else if (mesh->nn == 6 && ns == 2) ORD(6, 2);
  else if (mesh->nn == 4 && ns == 2) ORD(4, 2);
  else if (mesh->nn == 10 && ns == 2) ORD(10, 2);
  else if (mesh->nn == 10 && ns == 5) ORD(10, 5);
  else if (mesh->nn == 10 && ns == 1) ORD(10, 1);
  else if (mesh->nn == 8 && ns == 2) ORD(8, 2);
  else if (mesh->nn == 27 && ns == FA_Q2HEX_NSPLIT) ORD(27, FA_Q2HEX_NSPLIT);
  else if (mesh->nn == 64 && ns == FA_Q3HEX_NSPLIT) ORD(64, FA_Q3HEX_NSPLIT);
  else if (mesh->nn == 4 && ns == 1) ORD(4, 1);
  else if (mesh->nn == 9 && ns == 1) ORD(9, 1);
  else if (mesh->nn == 16 && ns == 4) ORD(16, 4);
  else ok = false;
#undef ORD
  if (src) HIP_TRY(hipFreeAsync(src, s));
  if (eperm) HIP_TRY(hipFreeAsync(eperm, s));
  if (!ok) return FA_OK;
  LAUNCH_CHECK();
  HIP_TRY(hipStreamSynchronize(s));
  plan->slot_order = ns;
  plan->eadj = posn ? eadj : nullptr;
  return FA_OK;
}

// Tensor cells: is every cell affine (x_v = x_0 + J xi_v at all vertices, J from vertices 1, 2, 4)?
// Sets *nonaffine when one is not (tolerance: 1e-12 of the cell's size).
template <int GD>
__global__ void k_check_affine(MeshView M, int* nonaffine) {
  constexpr int NV = 1 << GD;
  for (int64_t c = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; c < M.ncells; c += (int64_t)gridDim.x * blockDim.x) {
    const int32_t* g = M.geom + c * NV;
    double x[NV][GD];
#pragma unroll
    for (int v = 0; v < NV; ++v)
#pragma unroll
      for (int i = 0; i < GD; ++i) x[v][i] = M.x[(int64_t)g[v] * GD + i];
    double h = 0.0, dev = 0.0;
#pragma unroll
    for (int v = 1; v < NV; ++v)
#pragma unroll
      for (int i = 0; i < GD; ++i) {
        double pred = x[0][i];
#pragma unroll
        for (int k = 0; k < GD; ++k)
          if ((v >> k) & 1) pred += x[1 << k][i] - x[0][i];
        dev = fmax(dev, fabs(x[v][i] - pred));
        h = fmax(h, fabs(x[v][i] - x[0][i]));
      }
    if (dev > 1e-12 * h) atomicOr(nonaffine, 1);
  }
}

// plan_gather's device chunking: segment t = rows [rb0 + t * kChunkSeg, ...) cut greedily by one thread
// (a new chunk when the next row would exceed maxb blocks, maxadj entries or kGatherMaxRows rows; a row
// over a cap is reported), its starts at tmp[t * kChunkSeg + k], its count in cnt[t]
constexpr int64_t kChunkSeg = 2048;
__global__ void k_chunk_seg(const int64_t* __restrict__ ip, const int64_t* __restrict__ ap, int64_t rb0, int64_t n,
                            int64_t maxb, int maxadj, int64_t* __restrict__ tmp, int64_t* __restrict__ cnt,
                            int* __restrict__ st) {
  const int64_t nseg = (n - rb0 + kChunkSeg - 1) / kChunkSeg;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < nseg; t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r0 = rb0 + t * kChunkSeg, r1 = min(n, r0 + kChunkSeg);
    int64_t* out = tmp + t * kChunkSeg;
    int64_t k = 0, start = r0;
    int mb = 0, ma = 0, bad = INT32_MAX;
    int64_t ipr = ip[r0], apr = ap[r0], ips = ipr, aps = apr;
    out[k++] = r0;
    for (int64_t r = r0; r < r1; ++r) {
      const int64_t ipn = ip[r + 1], apn = ap[r + 1];
      if ((ipn - ipr > maxb || apn - apr > kGatherMaxAdj) && bad == INT32_MAX) bad = (int)(r - rb0);
      // maxadj is a target: a row with more entries gets a chunk of its own
      if (r > start && (ipn - ips > maxb || apn - aps > maxadj || r + 1 - start > kGatherMaxRows)) {
        out[k++] = r;
        mb = max(mb, (int)(ipr - ips));
        ma = max(ma, (int)(apr - aps));
        start = r;
        ips = ipr;
        aps = apr;
      }
      ipr = ipn;
      apr = apn;
    }
    mb = max(mb, (int)(ipr - ips));
    ma = max(ma, (int)(apr - aps));
    cnt[t] = k;
    atomicMax(&st[0], mb);
    atomicMax(&st[1], ma);
    if (bad != INT32_MAX) atomicMin(&st[2], bad);
  }
}
// row_start[off[t] + k] = tmp[t * kChunkSeg + k] for k < count of segment t; row_start[total] = n
__global__ void k_chunk_compact(const int64_t* __restrict__ tmp, const int64_t* __restrict__ off, int64_t rb0, int64_t n,
                                int64_t* __restrict__ row_start) {
  const int64_t nrows = n - rb0, nseg = (nrows + kChunkSeg - 1) / kChunkSeg;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nrows; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t t = i / kChunkSeg, k = i % kChunkSeg;
    if (off[t] + k < off[t + 1]) row_start[off[t] + k] = tmp[i];
    if (i == 0) row_start[off[nseg]] = n;
  }
}

// chunk rows so each chunk's blocks fit `maxb` accumulator blocks and its adjacency `maxadj`
static int plan_gather(const fa_mesh* mesh, const fa_adjacency* adj, const fa_bsr* A, int64_t* row_start,
                       fa_plan* plan, void* stream, int64_t maxb, int maxadj) {
  int rc = check_mesh(mesh);
  if (rc) return rc;
  if (!adj || !A || !row_start || !plan) return fail(FA_E_ARG, "null argument");
  hipStream_t s = (hipStream_t)stream;
  int64_t rb0 = A->row_begin, re0 = A->row_end;
  if (re0 <= rb0) { rb0 = 0; re0 = mesh->nnodes; }
  if (rb0 < 0 || re0 > mesh->nnodes) return fail(FA_E_ARG, "row window out of range");
  const int64_t n = re0;
  // Greedy chunking on the device (round 6; the host loop over config E's 67 M rows with their two
  // row pointer arrays copied to the host took 0.3-0.4 s of the plan): the window is cut into
  // segments of kChunkSeg rows, one thread each runs the greedy cut over its segment (a chunk always
  // starts at a segment's first row: one extra cut per kChunkSeg rows), then the per-segment starts
  // are compacted behind an exclusive scan of their counts.
  const int64_t nrows = n - rb0;
  const int64_t nseg = (nrows + kChunkSeg - 1) / kChunkSeg;  // 0 for an empty window
  int64_t* tmp = nullptr;   // [nrows] per-segment chunk starts (segment t at t * kChunkSeg)
  int64_t* cnt = nullptr;   // [nseg + 1] counts, then offsets
  int* st = nullptr;        // [4]: max blocks, max entries, first row over a cap (INT_MAX: none)
  void* scan_tmp = nullptr;
  size_t scan_bytes = 0;
  if ((rc = scratch_alloc((void**)&tmp, sizeof(int64_t) * (size_t)std::max<int64_t>(nrows, 1), s))) return rc;
  if ((rc = scratch_alloc((void**)&cnt, sizeof(int64_t) * (size_t)(nseg + 1), s))) return rc;
  if ((rc = scratch_alloc((void**)&st, sizeof(int) * 4, s))) return rc;
  static const int st0[4] = {0, 0, INT32_MAX, 0};
  HIP_TRY(hipMemcpyAsync(st, st0, sizeof(st0), hipMemcpyHostToDevice, s));
  HIP_TRY(hipMemsetAsync(cnt, 0, sizeof(int64_t) * (size_t)(nseg + 1), s));
  if (nseg > 0) {
    k_chunk_seg<<<grid_for(nseg, 64), 64, 0, s>>>(A->indptr, adj->ptr, rb0, n, maxb, maxadj, tmp, cnt, st);
    LAUNCH_CHECK();
  }
  HIP_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, scan_bytes, cnt, cnt, (int)(nseg + 1), s));
  if ((rc = scratch_alloc(&scan_tmp, std::max<size_t>(scan_bytes, 16), s))) return rc;
  HIP_TRY(hipcub::DeviceScan::ExclusiveSum(scan_tmp, scan_bytes, cnt, cnt, (int)(nseg + 1), s));
  if (nrows > 0) {
    k_chunk_compact<<<grid_for(nrows), 256, 0, s>>>(tmp, cnt, rb0, n, row_start);
    LAUNCH_CHECK();
  } else {
    HIP_TRY(hipMemcpyAsync(row_start, &rb0, sizeof(int64_t), hipMemcpyHostToDevice, s));
  }
  int64_t total = 0;
  int sth[3] = {0, 0, 0};
  HIP_TRY(hipMemcpyAsync(&total, cnt + nseg, sizeof(int64_t), hipMemcpyDeviceToHost, s));
  HIP_TRY(hipMemcpyAsync(sth, st, sizeof(int) * 3, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipFreeAsync(scan_tmp, s));
  HIP_TRY(hipFreeAsync(tmp, s));
  HIP_TRY(hipFreeAsync(cnt, s));
  HIP_TRY(hipFreeAsync(st, s));
  HIP_TRY(hipStreamSynchronize(s));
  if (sth[2] != INT32_MAX && sth[2] >= 0) {
    int64_t r = rb0 + sth[2], rp[2][2];
    HIP_TRY(hipMemcpy(rp[0], A->indptr + r, sizeof(int64_t) * 2, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(rp[1], adj->ptr + r, sizeof(int64_t) * 2, hipMemcpyDeviceToHost));
    return fail(FA_E_CAPACITY, "row %lld has %lld blocks / %lld cells (gather caps %lld / %d): use FA_SCATTER",
                (long long)r, (long long)(rp[0][1] - rp[0][0]), (long long)(rp[1][1] - rp[1][0]), (long long)maxb,
                kGatherMaxAdj);
  }
  const int32_t mb = sth[0], ma = sth[1];
  struct { int64_t k; int64_t size() const { return k; } } rs{total + 1};
  plan->nchunks = (int64_t)rs.size() - 1;
  plan->row_start = row_start;
  plan->cell_flags = 0;
  if ((mesh->cell_type == FA_HEXAHEDRON || mesh->cell_type == FA_QUADRILATERAL) && mesh->ncells > 0) {
    MeshView M{mesh->cells, mesh->geom, mesh->x, mesh->ncells, mesh->nnodes, mesh->nn, mesh->nv, mesh->gdim};
    int* dna = nullptr;
    int na_h = 1;
    HIP_TRY(hipMallocAsync((void**)&dna, sizeof(int), s));
    HIP_TRY(hipMemsetAsync(dna, 0, sizeof(int), s));
    if (mesh->gdim == 3) k_check_affine<3><<<grid_for(mesh->ncells), 256, 0, s>>>(M, dna);
    else k_check_affine<2><<<grid_for(mesh->ncells), 256, 0, s>>>(M, dna);
    LAUNCH_CHECK();
    HIP_TRY(hipMemcpyAsync(&na_h, dna, sizeof(int), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipFreeAsync(dna, s));
    HIP_TRY(hipStreamSynchronize(s));
    if (!na_h) plan->cell_flags |= FA_PLAN_AFFINE;
  }
  plan->max_blocks = mb;
  plan->max_adj = ma;
  plan->slots = nullptr;
  plan->slot_order = 0;
  plan->eadj = nullptr;
  plan->corder = nullptr;
  plan->contrib = nullptr;
  plan->chunk_desc = nullptr;
  return FA_OK;
}

extern "C" int fa_plan_gather(const fa_mesh* mesh, const fa_adjacency* adj, const fa_bsr* A, int64_t* row_start,
                              fa_plan* plan, void* stream) {
  if (!mesh) return fail(FA_E_ARG, "null mesh");
  int maxadj = std::min(FA_GATHER_ENTRY_CAP, kGatherMaxAdj);
  // simplices of the affine elasticity kernels: chunks of at most 256 items (k_gather_lin's one item
  // per lane), i.e. 256 / NSPLIT adjacency entries
  if (mesh->cell_type == FA_TRIANGLE || mesh->cell_type == FA_TETRAHEDRON) {
    DevTables T;
    int rc = get_tables(mesh->cell_type, mesh->degree, -1, &T);
    if (rc) return rc;
    const int ns = lin_simplex_nsplit(mesh->cell_type, mesh->degree, T.nq);
    if (ns > 0) {
      maxadj = std::min(maxadj, lin_threads(mesh->gdim, mesh->nn) / ns);
      return plan_gather(mesh, adj, A, row_start, plan, stream, lin_maxb(mesh->gdim, mesh->nn), maxadj);
    }
  }
  // quadrilaterals and Q1 hexahedra: k_gather_lin's caps too (affine cells of a packed table run it,
  // round 6; the generic gather of the others reads the same plan)
  if (mesh->cell_type == FA_QUADRILATERAL || (mesh->cell_type == FA_HEXAHEDRON && mesh->degree == 1)) {
    DevTables T;
    int rc = get_tables(mesh->cell_type, mesh->degree, -1, &T);
    if (rc) return rc;
    const int ns = lin_simplex_nsplit(mesh->cell_type, mesh->degree, T.nq, true);
    if (ns > 0 && T.pk) {
      maxadj = std::min(maxadj, lin_threads(mesh->gdim, mesh->nn) / ns);
      return plan_gather(mesh, adj, A, row_start, plan, stream, lin_maxb(mesh->gdim, mesh->nn), maxadj);
    }
  }
  return plan_gather(mesh, adj, A, row_start, plan, stream, gather_maxb(false, mesh->gdim * mesh->gdim), maxadj);
}

extern "C" int fa_plan_gather_form(const fa_mesh* mesh, int32_t kind, const fa_adjacency* adj, const fa_bsr* A,
                                   int64_t* row_start, fa_plan* plan, void* stream) {
  if (!mesh) return fail(FA_E_ARG, "null mesh");
  if (kind != FA_NEO_HOOKEAN) return fa_plan_gather(mesh, adj, A, row_start, plan, stream);
  const int rc = plan_gather(mesh, adj, A, row_start, plan, stream, gather_maxb(true, mesh->gdim * mesh->gdim),
                             256 / neo_nsplit(mesh->cell_type, mesh->degree));
  if (rc == FA_OK) plan->cell_flags |= FA_PLAN_NEO;
  return rc;
}

// ------------------------------------------------------------------------------- contribution plan
static inline int64_t align256(int64_t b);
__global__ void k_chunk_desc(const int64_t* __restrict__ row_start, int64_t nchunks, const int64_t* __restrict__ indptr,
                             const int64_t* __restrict__ adj_ptr, int64_t* __restrict__ cb, int64_t* __restrict__ ca);
// Chunking for k_gather_own: its output staging holds own_maxb blocks and its record staging
// FA_OWN_CCAP cells (<= adjacency entries of the chunk).
extern "C" int fa_plan_gather_contrib(const fa_mesh* mesh, const fa_adjacency* adj, const fa_bsr* A,
                                      int64_t* row_start, fa_plan* plan, void* stream) {
  if (!mesh) return fail(FA_E_ARG, "null mesh");
  return plan_gather(mesh, adj, A, row_start, plan, stream, own_maxb(mesh->gdim * mesh->gdim), FA_OWN_CCAP);
}

// One workgroup per chunk. For entry j (row node a of cell c) and column node b: the block's
// chunk position p (search of the column in the row's pattern) and its rank among the row's
// earlier entries whose cell also holds that column (a deterministic order within the block);
// counting sort by p; contribution i of the sorted list goes to lane i / K, word i % K.
template <int NN>
__global__ __launch_bounds__(256) void k_plan_contrib(const int32_t* __restrict__ dofmap, const int64_t* __restrict__ row_start,
                                                      int64_t nchunks, const int64_t* __restrict__ indptr,
                                                      const int32_t* __restrict__ indices, const int64_t* __restrict__ adj_ptr,
                                                      const int32_t* __restrict__ adj_idx, const int64_t* __restrict__ cw,
                                                      int32_t* __restrict__ ccells, uint16_t* __restrict__ words, int maxb,
                                                      int* err) {
  constexpr int CCAP = FA_OWN_CCAP, NC = CCAP * NN;
  __shared__ int32_t s_cols[1024];
  __shared__ int32_t s_cnt[1024], s_start[1024];
  __shared__ int32_t s_rowoff[kGatherMaxRows + 1], s_eoff[kGatherMaxRows + 1];
  __shared__ int32_t s_ent[CCAP], s_first[CCAP];
  __shared__ uint8_t s_erow[CCAP], s_eslot[CCAP];
  __shared__ int32_t s_dofs[NC];
  __shared__ int16_t s_pos[NC], s_rank[NC], s_inv[NC];
  __shared__ int s_nslot;
  const int tid = threadIdx.x;
  for (int64_t c = blockIdx.x; c < nchunks; c += gridDim.x) {
    const int64_t r0 = row_start[c], r1 = row_start[c + 1];
    const int64_t b0 = indptr[r0], b1 = indptr[r1], a0 = adj_ptr[r0], a1 = adj_ptr[r1];
    const int nr = (int)(r1 - r0), nb = (int)(b1 - b0), na = (int)(a1 - a0);
    if (nr > kGatherMaxRows || nb > maxb || nb > 1024 || na > CCAP) {
      if (tid == 0) atomicOr(err, 1);
      continue;  // uniform over the workgroup
    }
    const int n = na * NN;
    const int K = (int)((cw[c + 1] - cw[c]) >> 8) - 1;
    uint16_t* wp = words + cw[c];
    for (int t = tid; t < nb; t += 256) {
      s_cols[t] = indices[b0 + t];
      s_cnt[t] = 0;
    }
    if (tid <= nr) {
      s_rowoff[tid] = (int)(indptr[r0 + tid] - b0);
      s_eoff[tid] = (int)(adj_ptr[r0 + tid] - a0);
    }
    if (tid < na) s_ent[tid] = adj_idx[a0 + tid];
    __syncthreads();
    if (tid < nr)
      for (int j = s_eoff[tid]; j < s_eoff[tid + 1]; ++j) s_erow[j] = (uint8_t)tid;
    for (int t = tid; t < n; t += 256) s_dofs[t] = dofmap[(int64_t)(s_ent[t / NN] / NN) * NN + t % NN];
    if (tid < na) {  // first entry of the chunk with this entry's cell
      const int cell = s_ent[tid] / NN;
      int f = tid;
      for (int j = 0; j < tid; ++j)
        if (s_ent[j] / NN == cell) { f = j; break; }
      s_first[tid] = f;
    }
    __syncthreads();
    if (tid < na) {  // the cell's slot: distinct cells in order of first appearance
      const int f = s_first[tid];
      int sl = 0;
      for (int j = 0; j < f; ++j) sl += s_first[j] == j;
      s_eslot[tid] = (uint8_t)sl;
      if (f == tid) ccells[c * CCAP + sl] = s_ent[tid] / NN;
    }
    if (tid == 0) {
      int ns = 0;
      for (int j = 0; j < na; ++j) ns += s_first[j] == j;
      s_nslot = ns;
    }
    for (int t = tid; t < n; t += 256) {
      const int j = t / NN, row = s_erow[j];
      const int32_t col = s_dofs[t];
      int p = lds_find(s_cols, s_rowoff[row], s_rowoff[row + 1], col);
      if (p < 0) {
        atomicOr(err, 2);
        p = 0;
      }
      s_pos[t] = (int16_t)p;
      atomicAdd(&s_cnt[p], 1);
      int rk = 0;
      for (int j2 = s_eoff[row]; j2 < j; ++j2)
        for (int bb = 0; bb < NN; ++bb)
          if (s_dofs[j2 * NN + bb] == col) { ++rk; break; }
      s_rank[t] = (int16_t)rk;
    }
    __syncthreads();
    if (tid == 0) {
      int acc = 0;
      for (int p = 0; p < nb; ++p) {
        s_start[p] = acc;
        if (s_cnt[p] == 0) atomicOr(err, 4);  // a pattern block no cell contributes to
        acc += s_cnt[p];
      }
    }
    if (tid < CCAP && tid >= s_nslot) ccells[c * CCAP + tid] = -1;
    __syncthreads();
    for (int t = tid; t < n; t += 256) {
      const int p = s_pos[t], rk = s_rank[t];
      const int i = s_start[p] + rk;
      const int lane = i / K, k = i - lane * K;
      const int j = t / NN, b = t % NN, a = s_ent[j] % NN;
      const uint32_t w = (uint32_t)s_eslot[j] | ((uint32_t)(a * NN + b) << 8) | (rk == s_cnt[p] - 1 ? 0x8000u : 0u);
      wp[256 + k * 256 + lane] = (uint16_t)w;
      s_inv[i] = (int16_t)t;
    }
    for (int i = n + tid; i < K * 256; i += 256) {
      const int lane = i / K, k = i - lane * K;
      wp[256 + k * 256 + lane] = (uint16_t)kOwnPad;
    }
    __syncthreads();
    {
      const int i = tid * K;
      wp[tid] = (uint16_t)(i < n ? (uint32_t)s_pos[s_inv[i]] : kOwnIdle);
    }
    __syncthreads();
  }
}

// word-section offsets of a plan's chunks (u16 units): 256 lane starts + K x 256 words, K =
// ceil(nn * entries / 256); *bytes = the whole buffer [cw | ccells | words]
static int contrib_layout(const fa_mesh* mesh, const fa_adjacency* adj, const fa_bsr* A, const fa_plan* plan, hipStream_t s,
                          std::vector<int64_t>& cw, int64_t* bytes) {
  int rc = check_mesh(mesh);
  if (rc) return rc;
  if (!adj || !A || !plan || !plan->row_start) return fail(FA_E_ARG, "null argument");
  const int64_t nch = plan->nchunks;
  if (nch >= (1ll << 31)) return fail(FA_E_CAPACITY, "contribution plan: %lld chunks", (long long)nch);
  int64_t* d = nullptr;
  HIP_TRY(hipMallocAsync((void**)&d, sizeof(int64_t) * 2 * (nch + 1), s));
  k_chunk_desc<<<grid_for(nch + 1), 256, 0, s>>>(plan->row_start, nch, A->indptr, adj->ptr, d, d + nch + 1);
  LAUNCH_CHECK();
  std::vector<int64_t> ca(nch + 1);
  HIP_TRY(hipMemcpyAsync(ca.data(), d + nch + 1, sizeof(int64_t) * (nch + 1), hipMemcpyDeviceToHost, s));
  HIP_TRY(hipFreeAsync(d, s));
  HIP_TRY(hipStreamSynchronize(s));
  cw.assign(nch + 1, 0);
  for (int64_t c = 0; c < nch; ++c) {
    const int64_t n = (ca[c + 1] - ca[c]) * mesh->nn;
    cw[c + 1] = cw[c] + 256 * ((n + 255) / 256 + 1);
  }
  *bytes = align256(8 * (nch + 1)) + align256(4 * nch * (int64_t)FA_OWN_CCAP) + align256(2 * cw[nch]);
  return FA_OK;
}

static bool contrib_element(const fa_mesh* m) {
  return (m->cell_type == FA_TRIANGLE || m->cell_type == FA_TETRAHEDRON) && (m->degree == 1 || m->degree == 2);
}

extern "C" int fa_plan_contrib_bytes(const fa_mesh* mesh, const fa_adjacency* adj, const fa_bsr* A, const fa_plan* plan,
                                     int64_t* bytes, void* stream) {
  if (!bytes) return fail(FA_E_ARG, "null bytes");
  std::vector<int64_t> cw;
  return contrib_layout(mesh, adj, A, plan, (hipStream_t)stream, cw, bytes);
}

extern "C" int fa_plan_contrib(const fa_mesh* mesh, const fa_adjacency* adj, const fa_bsr* A, void* buf, int64_t bytes,
                               fa_plan* plan, void* stream) {
  int rc = check_mesh(mesh);
  if (rc) return rc;
  if (!plan || !buf) return fail(FA_E_ARG, "null argument");
  plan->contrib = nullptr;
  if (!contrib_element(mesh)) return fail(FA_E_UNSUPPORTED, "contribution plans serve P1/P2 triangles and tetrahedra");
  const int bs2 = mesh->gdim * mesh->gdim;
  if (plan->max_blocks > own_maxb(bs2) || plan->max_adj > FA_OWN_CCAP)
    return fail(FA_E_CAPACITY, "plan chunks hold %d blocks / %d entries (contribution kernel: %d / %d): plan with "
                "fa_plan_gather_contrib", plan->max_blocks, plan->max_adj, own_maxb(bs2), FA_OWN_CCAP);
  hipStream_t s = (hipStream_t)stream;
  std::vector<int64_t> cw;
  int64_t need = 0;
  if ((rc = contrib_layout(mesh, adj, A, plan, s, cw, &need))) return rc;
  if (bytes < need) return fail(FA_E_ARG, "contribution buffer holds %lld bytes, the plan needs %lld", (long long)bytes,
                                (long long)need);
  const int64_t nch = plan->nchunks;
  char* base = static_cast<char*>(buf);
  int64_t* dcw = reinterpret_cast<int64_t*>(base);
  int32_t* dcells = reinterpret_cast<int32_t*>(base + align256(8 * (nch + 1)));
  uint16_t* dwords = reinterpret_cast<uint16_t*>(base + align256(8 * (nch + 1)) + align256(4 * nch * (int64_t)FA_OWN_CCAP));
  HIP_TRY(hipMemcpyAsync(dcw, cw.data(), sizeof(int64_t) * (nch + 1), hipMemcpyHostToDevice, s));
  int* derr = nullptr;
  HIP_TRY(hipMallocAsync((void**)&derr, sizeof(int), s));
  HIP_TRY(hipMemsetAsync(derr, 0, sizeof(int), s));
  const int grid = (int)std::min<int64_t>(std::max<int64_t>(nch, 1), 1 << 20);
  switch (mesh->nn) {
    case 3: k_plan_contrib<3><<<grid, 256, 0, s>>>(mesh->cells, plan->row_start, nch, A->indptr, A->indices, adj->ptr, adj->idx, dcw, dcells, dwords, own_maxb(bs2), derr); break;
    case 6: k_plan_contrib<6><<<grid, 256, 0, s>>>(mesh->cells, plan->row_start, nch, A->indptr, A->indices, adj->ptr, adj->idx, dcw, dcells, dwords, own_maxb(bs2), derr); break;
    case 4: k_plan_contrib<4><<<grid, 256, 0, s>>>(mesh->cells, plan->row_start, nch, A->indptr, A->indices, adj->ptr, adj->idx, dcw, dcells, dwords, own_maxb(bs2), derr); break;
    case 10: k_plan_contrib<10><<<grid, 256, 0, s>>>(mesh->cells, plan->row_start, nch, A->indptr, A->indices, adj->ptr, adj->idx, dcw, dcells, dwords, own_maxb(bs2), derr); break;
    default: (void)hipFreeAsync(derr, s); return fail(FA_E_UNSUPPORTED, "contribution plan: %d nodes per cell", mesh->nn);
  }
  LAUNCH_CHECK();
  int herr = 0;
  HIP_TRY(hipMemcpyAsync(&herr, derr, sizeof(int), hipMemcpyDeviceToHost, s));
  HIP_TRY(hipFreeAsync(derr, s));
  HIP_TRY(hipStreamSynchronize(s));
  if (herr) return fail(FA_E_PATTERN, "contribution plan: chunk capacity / pattern error 0x%x", herr);
  plan->contrib = buf;
  return FA_OK;
}

// the kernel's views of plan->contrib (NULL pointers without one)
static void set_contrib(GatherArgs& P, const fa_plan* plan) {
  P.cw = nullptr;
  P.ccells = nullptr;
  P.cwords = nullptr;
  if (!plan || !plan->contrib) return;
  const int64_t nch = plan->nchunks;
  const char* base = static_cast<const char*>(plan->contrib);
  P.cw = reinterpret_cast<const int64_t*>(base);
  P.ccells = reinterpret_cast<const int32_t*>(base + align256(8 * (nch + 1)));
  P.cwords = reinterpret_cast<const uint16_t*>(base + align256(8 * (nch + 1)) + align256(4 * nch * (int64_t)FA_OWN_CCAP));
}

// ------------------------------------------------------------------------------- chunk locality order
static int scratch_alloc(void** p, size_t bytes, hipStream_t s);
static inline int64_t align256(int64_t b);
// Doubles <-> order-preserving unsigned keys (for atomic min / max of coordinates).
__device__ inline unsigned long long ordered_key(double v) {
  const unsigned long long b = (unsigned long long)__double_as_longlong(v);
  return (b >> 63) ? ~b : (b | (1ull << 63));
}
__device__ inline double ordered_val(unsigned long long k) {
  return __longlong_as_double((long long)((k >> 63) ? (k & ~(1ull << 63)) : ~k));
}
// a point per chunk: the centroid of the cell of the chunk's first adjacency entry; bounding box
// of the points in bb[0..2] (min keys) / bb[3..5] (max keys), one atomic per workgroup and axis
__global__ __launch_bounds__(256) void k_chunk_points(MeshView M, const int64_t* __restrict__ row_start, int64_t nchunks,
                                                      const int64_t* __restrict__ adj_ptr,
                                                      const int32_t* __restrict__ adj_idx, double* __restrict__ pts,
                                                      unsigned long long* __restrict__ bb) {
  __shared__ unsigned long long smin[3][256], smax[3][256];
  unsigned long long lmin[3] = {~0ull, ~0ull, ~0ull}, lmax[3] = {0ull, 0ull, 0ull};
  for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < nchunks; k += (int64_t)gridDim.x * blockDim.x) {
    const int64_t e = adj_ptr[row_start[k]];
    double p[3] = {0.0, 0.0, 0.0};
    // a chunk whose rows touch no cell (unused nodes) has no entry to locate it: it keeps the
    // origin as its point (any order assembles the same matrix)
    const bool has = e < adj_ptr[row_start[k + 1]];
    if (has) {
      const int64_t c = adj_idx[e] / M.nn;
      for (int v = 0; v < M.nv; ++v)
        for (int i = 0; i < M.gd; ++i) p[i] += M.x[(int64_t)M.geom[c * M.nv + v] * M.gd + i];
    }
    for (int i = 0; i < 3; ++i) {
      p[i] = has ? p[i] / (double)M.nv : 0.0;
      pts[k * 3 + i] = p[i];
      const unsigned long long q = ordered_key(p[i]);
      lmin[i] = min(lmin[i], q);
      lmax[i] = max(lmax[i], q);
    }
  }
  for (int i = 0; i < 3; ++i) {
    smin[i][threadIdx.x] = lmin[i];
    smax[i][threadIdx.x] = lmax[i];
  }
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w)
      for (int i = 0; i < 3; ++i) {
        smin[i][threadIdx.x] = min(smin[i][threadIdx.x], smin[i][threadIdx.x + w]);
        smax[i][threadIdx.x] = max(smax[i][threadIdx.x], smax[i][threadIdx.x + w]);
      }
    __syncthreads();
  }
  if (threadIdx.x < 3) {
    atomicMin(bb + threadIdx.x, smin[threadIdx.x][0]);
    atomicMax(bb + 3 + threadIdx.x, smax[threadIdx.x][0]);
  }
}
__device__ inline uint64_t spread3(uint64_t v) {  // 21 bits -> every third bit
  v &= 0x1fffffull;
  v = (v | (v << 32)) & 0x1f00000000ffffull;
  v = (v | (v << 16)) & 0x1f0000ff0000ffull;
  v = (v | (v << 8)) & 0x100f00f00f00f00full;
  v = (v | (v << 4)) & 0x10c30c30c30c30c3ull;
  v = (v | (v << 2)) & 0x1249249249249249ull;
  return v;
}
__global__ void k_chunk_morton(const double* __restrict__ pts, int64_t nchunks, const unsigned long long* __restrict__ bb,
                               uint64_t* __restrict__ keys, int32_t* __restrict__ vals) {
  for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < nchunks; k += (int64_t)gridDim.x * blockDim.x) {
    uint64_t key = 0;
    for (int i = 0; i < 3; ++i) {
      const double lo = ordered_val(bb[i]), hi = ordered_val(bb[3 + i]);
      const double t = hi > lo ? (pts[k * 3 + i] - lo) / (hi - lo) : 0.0;
      const uint64_t q = (uint64_t)fmin(fmax(t * 2097152.0, 0.0), 2097151.0);
      key |= spread3(q) << i;
    }
    keys[k] = key;
    vals[k] = (int32_t)k;
  }
}

extern "C" int fa_plan_locality(const fa_mesh* mesh, const fa_adjacency* adj, int32_t* corder, fa_plan* plan,
                                void* stream) {
  int rc = check_mesh(mesh);
  if (rc) return rc;
  if (!adj || !adj->ptr || !adj->idx || !corder || !plan || !plan->row_start) return fail(FA_E_ARG, "null argument");
  plan->chunk_desc = nullptr;  // built for the previous order
  hipStream_t s = (hipStream_t)stream;
  const int64_t n = plan->nchunks;
  if (n >= (1ll << 31)) return fail(FA_E_CAPACITY, "gather plan has %lld chunks (>= 2^31)", (long long)n);
  if (n <= 1 || mesh->ncells == 0) {
    plan->corder = nullptr;
    return FA_OK;
  }
  MeshView M{mesh->cells, mesh->geom, mesh->x, mesh->ncells, mesh->nnodes, mesh->nn, mesh->nv, mesh->gdim};
  // scratch: points [n][3] f64, bbox 6 keys, keys in/out u64, vals in i32, radix-sort temp
  size_t temp_bytes = 0;
  HIP_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, temp_bytes, (uint64_t*)nullptr, (uint64_t*)nullptr,
                                             (int32_t*)nullptr, (int32_t*)nullptr, (int)n, 0, 63, s));
  const size_t off_bb = align256(sizeof(double) * 3 * n);
  const size_t off_k0 = off_bb + 256;
  const size_t off_k1 = off_k0 + align256(sizeof(uint64_t) * n);
  const size_t off_v = off_k1 + align256(sizeof(uint64_t) * n);
  const size_t off_t = off_v + align256(sizeof(int32_t) * n);
  char* buf = nullptr;
  if ((rc = scratch_alloc((void**)&buf, off_t + temp_bytes, s))) return rc;
  double* pts = reinterpret_cast<double*>(buf);
  unsigned long long* bb = reinterpret_cast<unsigned long long*>(buf + off_bb);
  uint64_t* k0 = reinterpret_cast<uint64_t*>(buf + off_k0);
  uint64_t* k1 = reinterpret_cast<uint64_t*>(buf + off_k1);
  int32_t* v0 = reinterpret_cast<int32_t*>(buf + off_v);
  const unsigned long long init[6] = {~0ull, ~0ull, ~0ull, 0ull, 0ull, 0ull};
  HIP_TRY(hipMemcpyAsync(bb, init, sizeof(init), hipMemcpyHostToDevice, s));
  k_chunk_points<<<grid_for(n), 256, 0, s>>>(M, plan->row_start, n, adj->ptr, adj->idx, pts, bb);
  LAUNCH_CHECK();
  k_chunk_morton<<<grid_for(n), 256, 0, s>>>(pts, n, bb, k0, v0);
  LAUNCH_CHECK();
  HIP_TRY(hipcub::DeviceRadixSort::SortPairs(buf + off_t, temp_bytes, k0, k1, v0, corder, (int)n, 0, 63, s));
  HIP_TRY(hipFreeAsync(buf, s));
  HIP_TRY(hipStreamSynchronize(s));
  plan->corder = corder;
  return FA_OK;
}

// The plan's chunk arrays once (fa_plan_chunk_desc): k_lin_chunk_desc as a launch would run it, into a
// caller-owned buffer kept with the plan.
__global__ void k_lin_chunk_desc(const int64_t* __restrict__ row_start, int64_t nchunks, const int64_t* __restrict__ indptr,
                                 int64_t row_begin, const int64_t* __restrict__ adj_ptr, int64_t nent,
                                 const int32_t* __restrict__ seq, int64_t* __restrict__ cb, int64_t* __restrict__ ca);
extern "C" int fa_plan_chunk_desc(const fa_mesh* mesh, const fa_adjacency* adj, const fa_bsr* A, fa_plan* plan,
                                  int64_t* buf, void* stream) {
  int rc = check_mesh(mesh);
  if (rc) return rc;
  if (!adj || !adj->ptr || !A || !A->indptr || !plan || !plan->row_start || !buf) return fail(FA_E_ARG, "null argument");
  if (plan->nchunks >= (1ll << 30)) return fail(FA_E_CAPACITY, "gather plan has %lld chunks (>= 2^30)", (long long)plan->nchunks);
  int64_t wb = A->row_begin, we = A->row_end;
  if (we <= wb) { wb = 0; we = mesh->nnodes; }
  if (wb < 0 || we > mesh->nnodes) return fail(FA_E_ARG, "row window out of range");
  hipStream_t s = (hipStream_t)stream;
  plan->chunk_desc = nullptr;
  if (plan->nchunks > 0) {
    k_lin_chunk_desc<<<grid_for(plan->nchunks), 256, 0, s>>>(plan->row_start, plan->nchunks, A->indptr, wb, adj->ptr,
                                                             mesh->ncells * mesh->nn, plan->corder, buf,
                                                             buf + (plan->nchunks + 1));
    LAUNCH_CHECK();
  }
  plan->chunk_desc = buf;
  return FA_OK;
}

// ------------------------------------------------------------------------------------ assemble_matrix
static int form_view(const fa_mesh* mesh, const fa_form* form, FormView& F) {
  if (!form) return fail(FA_E_ARG, "null form");
  F.kind = form->kind;
  F.ad = 0;
  if (F.kind == FA_ASYM_DAMAGE_AD) {  // the damage law with the USE_AD tangent and stress
    F.kind = FA_ASYM_DAMAGE;
    F.ad = 1;
  }
  F.E = form->E;
  F.nu = form->nu;
  F.lam = form->lam;
  F.mu = form->mu;
  F.u = form->u;
  F.d = form->d;
  F.f = form->f;
  if (!F.E && (!F.lam || !F.mu)) return fail(FA_E_ARG, "form needs E (+nu) or lam and mu");
  if (F.kind == FA_ASYM_DAMAGE) {
    if (mesh->cell_type != FA_TRIANGLE || mesh->degree != 1)
      return fail(FA_E_UNSUPPORTED, "FA_ASYM_DAMAGE is the reference's 2-D P1-triangle law");
  } else if (F.kind == FA_NEO_HOOKEAN) {
    if (!F.u) return fail(FA_E_ARG, "FA_NEO_HOOKEAN needs the state u");
  } else if (F.kind != FA_LINEAR_ELASTICITY) {
    return fail(FA_E_UNSUPPORTED, "form kind %d not implemented", F.kind);
  }
  return FA_OK;
}

// scratch for per-cell records: stream-ordered, from a pool that keeps its memory
static int scratch_alloc(void** p, size_t bytes, hipStream_t s) {
  static bool pool_set = false;
  if (!pool_set) {
    int dev = 0;
    hipMemPool_t pool;
    if (hipGetDevice(&dev) == hipSuccess && hipDeviceGetDefaultMemPool(&pool, dev) == hipSuccess) {
      uint64_t thr = UINT64_MAX;
      (void)hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &thr);
    }
    pool_set = true;
  }
  HIP_TRY(hipMallocAsync(p, bytes > 0 ? bytes : 16, s));
  return FA_OK;
}

// per-chunk block / adjacency offsets: one dependent load level less in the gather's pipeline
__global__ void k_chunk_desc(const int64_t* __restrict__ row_start, int64_t nchunks, const int64_t* __restrict__ indptr,
                             const int64_t* __restrict__ adj_ptr, int64_t* __restrict__ cb, int64_t* __restrict__ ca) {
  for (int64_t c = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; c <= nchunks; c += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = row_start[c];
    cb[c] = indptr[r];
    ca[c] = adj_ptr[r];
  }
}

static int chunk_desc(GatherArgs& P, int64_t** buf, hipStream_t s) {
  int rc;
  if (P.nchunks >= (1ll << 31)) return fail(FA_E_CAPACITY, "gather plan has %lld chunks (>= 2^31)", (long long)P.nchunks);
  if ((rc = scratch_alloc((void**)buf, sizeof(int64_t) * (2 * (P.nchunks + 1) + 8), s))) return rc;
  P.chunk_b = *buf;
  P.chunk_a = *buf + (P.nchunks + 1);
  P.ctr = reinterpret_cast<unsigned long long*>(*buf + 2 * (P.nchunks + 1));
  HIP_TRY(hipMemsetAsync(P.ctr, 0, 8 * sizeof(unsigned long long), s));
  k_chunk_desc<<<grid_for(P.nchunks + 1), 256, 0, s>>>(P.row_start, P.nchunks, P.A.indptr, P.adj_ptr, *buf,
                                                      *buf + (P.nchunks + 1));
  LAUNCH_CHECK();
  return FA_OK;
}

// k_gather_lin's chunk arrays: per chunk c, chunk_b[c] = its first block relative to the window,
// chunk_a[c] = its first adjacency entry (clamped below the entry count, so a lane's entry load is
// always in range) and chunk_a[nchunks + 1 + c] = block count | entry count << 32: three scalar
// loads per chunk, no dependent level, and fewer pointers live in the kernel's loop
// Position i of the arrays describes chunk seq[i] (the plan's visiting order) or chunk i (seq NULL).
__global__ void k_lin_chunk_desc(const int64_t* __restrict__ row_start, int64_t nchunks, const int64_t* __restrict__ indptr,
                                 int64_t row_begin, const int64_t* __restrict__ adj_ptr, int64_t nent,
                                 const int32_t* __restrict__ seq, int64_t* __restrict__ cb, int64_t* __restrict__ ca) {
  const int64_t base = indptr[row_begin];
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nchunks; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t c = seq ? (int64_t)seq[i] : i;
    const int64_t r0 = row_start[c], r1 = row_start[c + 1];
    const int64_t b0 = indptr[r0], a0 = adj_ptr[r0];
    cb[i] = b0 - base;
    ca[i] = min(a0, max(nent - 1, (int64_t)0));
    ca[nchunks + 1 + i] = (int64_t)((uint64_t)(uint32_t)(indptr[r1] - b0) | ((uint64_t)(uint32_t)(adj_ptr[r1] - a0) << 32));
  }
}

// the chunk arrays of the persistent per-XCD schedule (k_gather_lin, k_gather_neo) in the order seq
// (NULL: row order), and the XCD counters (zeroed)
static int lin_chunk_desc(GatherArgs& P, int64_t** buf, hipStream_t s, const int32_t* seq) {
  int rc;
  if (P.nchunks >= (1ll << 30)) return fail(FA_E_CAPACITY, "gather plan has %lld chunks (>= 2^30)", (long long)P.nchunks);
  if (P.chunk_desc) {  // the plan's arrays (fa_plan_chunk_desc): only the XCD counters per launch
    if ((rc = scratch_alloc((void**)buf, 1024, s))) return rc;
    P.chunk_b = P.chunk_desc;
    P.chunk_a = P.chunk_desc + (P.nchunks + 1);
    P.ctr = reinterpret_cast<unsigned long long*>(*buf);
    HIP_TRY(hipMemsetAsync(P.ctr, 0, 1024, s));
    return FA_OK;
  }
  if ((rc = scratch_alloc((void**)buf, sizeof(int64_t) * (3 * (P.nchunks + 1) + 128), s))) return rc;
  P.chunk_b = *buf;
  P.chunk_a = *buf + (P.nchunks + 1);
  P.ctr = reinterpret_cast<unsigned long long*>(*buf + 3 * (P.nchunks + 1));  // 8 counters, 128 B apart
  HIP_TRY(hipMemsetAsync(P.ctr, 0, 1024, s));
  k_lin_chunk_desc<<<grid_for(P.nchunks), 256, 0, s>>>(P.row_start, P.nchunks, P.A.indptr, P.A.row_begin, P.adj_ptr,
                                                       P.M.ncells * P.M.nn, seq, *buf, *buf + (P.nchunks + 1));
  LAUNCH_CHECK();
  return FA_OK;
}

// Gather grid. Default (dynamic): a persistent grid of the resident workgroup count (CUs x
// occupancy, a multiple of 8 for the XCD order), each workgroup pulling chunks from its XCD's
// counter with three chunks of look-ahead, so chunk k's stores, chunk k+1's metadata loads and
// the per-workgroup LDS tables overlap the work instead of heading every chunk (measured on
// config E: skeleton 41.9 -> 33.0 ms persistent; a static grid of one workgroup per chunk, and
// larger persistent grids, measured slower).
template <typename K>
static int64_t gather_grid(K kernel, int64_t nchunks, int block = 256) {
  const int64_t per = (nchunks + 7) / 8;
  int dev = 0, cus = 256, occ = 4;
  if (hipGetDevice(&dev) == hipSuccess) {
    int v = 0;
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0) cus = v;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&v, kernel, block, 0) == hipSuccess && v > 0) occ = v;
  }
  int64_t g = (int64_t)cus * occ;
  g = std::max<int64_t>(8, g / 8 * 8);
  return std::min<int64_t>(std::min<int64_t>(8 * per, g), kMaxBlocks);  // kMaxBlocks % 8 == 0
}

// What a gather launch does: both stages with stream-ordered scratch (fa_assemble_matrix), or
// one stage on a caller-owned work buffer (fa_gather_prepare / fa_gather_rows), or only report
// that buffer's size.
struct GatherStage {
  enum { FULL, SIZE, PREP, ROWS } mode = FULL;
  void* work = nullptr;
  int64_t* bytes = nullptr;
};
static inline int64_t align256(int64_t b) { return (b + 255) & ~int64_t(255); }

// every node's coordinates and constrained-dof bits (bit j: dof node * GD + j), for the fused P1 records
template <int GD>
__global__ void k_pack_nodes(const double* __restrict__ x, const int8_t* __restrict__ bc, int64_t nnodes,
                             double* __restrict__ out) {
  // node n -> {x, y, z, bits} (GD = 3) or {x, y, bits, 0} (GD = 2): one vertex in two 16-B loads of
  // the fused gather (its coordinates were GD 8-B loads and its bc bits a byte load), round 5
  for (int64_t n = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; n < nnodes; n += (int64_t)gridDim.x * blockDim.x) {
    uint32_t m = 0u;
    if (bc) {
#pragma unroll
      for (int j = 0; j < GD; ++j) m |= (bc[n * GD + j] ? 1u : 0u) << j;
    }
    const double mb = __longlong_as_double((long long)m);
    const fa_dv2 a = fa_dv2{x[n * GD], x[n * GD + 1]};
    const fa_dv2 b = GD == 3 ? fa_dv2{x[n * GD + GD - 1], mb} : fa_dv2{mb, 0.0};
    fa_dv2* o = reinterpret_cast<fa_dv2*>(out + 4 * n);
    o[0] = a;
    store_guard1(a);
    o[1] = b;
    store_guard1(b);
  }
}

template <int GD>
__global__ void k_bhat(const double* __restrict__ ahat, int nblk, double r, double* __restrict__ bhat) {
  for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < nblk; t += gridDim.x * blockDim.x) {
    double o[GD * GD];
#pragma unroll
    for (int i = 0; i < GD; ++i)
#pragma unroll
      for (int k = 0; k < GD; ++k) o[i * GD + k] = r * ahat[t * GD * GD + i * GD + k] + ahat[t * GD * GD + k * GD + i];
#pragma unroll
    for (int e = 0; e < GD * GD; ++e) bhat[t * GD * GD + e] = o[e];
    store_fence(o);
  }
}

// k_gather_lin's constant operands: a zero mask word (no bcs) and a scratch line for the stores of
// a chunk without values; allocated once per process
static int lin_scratch(uint32_t** zero32, double** dump) {
  static uint32_t* z = nullptr;
  static double* d = nullptr;
  static std::mutex mu;
  std::lock_guard<std::mutex> lk(mu);
  if (!z) {
    void* p = nullptr;
    HIP_TRY(hipMalloc(&p, 4096));
    HIP_TRY(hipMemset(p, 0, 4096));
    z = reinterpret_cast<uint32_t*>(p);
    d = reinterpret_cast<double*>(reinterpret_cast<char*>(p) + 256);
  }
  *zero32 = z;
  *dump = d;
  return FA_OK;
}

// FIX bound constant of k_gather_lin: |block entry| <= fixc * rho^2, rho = sum |s Ji| of the record.
// P1 blocks (from the record's gradients g, |g_i| <= rho): cv (|r| g_a g_b^T + g_b g_a^T + (g_a.g_b) I);
// table blocks: (s Ji)^T B (s Ji) + tr / (1 + r) I with |B| <= (|r| + 1) amax
static double lin_fix_bound(int gd, int nn, double rlm, double trc, double amax) {
  if (nn == gd + 1) return (gd == 2 ? 0.5 : 1.0 / 6.0) * (std::fabs(rlm) + 1.0 + gd);
  return (std::fabs(rlm) + 1.0) * amax * (1.0 + gd * std::fabs(trc));
}

static bool neo_m_plan_ok(const GatherArgs& P, int nsplit) {
  return P.eadj && P.slots && P.slot_order == nsplit && !P.cw && P.plan_maxadj >= 0 && P.plan_maxadj * nsplit <= 256;
}

template <int GD, int NN, int NQ, int NSPLIT>
static int launch_gather_neo(GatherArgs P, const int8_t* bc, hipStream_t s, const GatherStage& W) {
  using R = NeoM<GD, NQ>;
  const int64_t nc = P.M.ncells;
  const int64_t rec_bytes = align256((int64_t)sizeof(double) * R::count(nc));
  if (W.mode == GatherStage::SIZE) {
    *W.bytes = rec_bytes + align256((int64_t)sizeof(uint32_t) * nc);
    return FA_OK;
  }
  const bool rows = P.nchunks > 0 && W.mode != GatherStage::PREP;
  if (rows && P.fix) return fail(FA_E_UNSUPPORTED, "deterministic assembly: not for the neo-Hookean gather");
  if (rows) {  // the kernel's plan: positional, ordered for NSPLIT, <= 256 items per chunk
    if (!neo_m_plan_ok(P, NSPLIT))
      return fail(FA_E_ARG, "the neo-Hookean gather needs a positional plan ordered for %d column parts with <= %d "
                  "entries per chunk (fa_plan_gather_form + fa_plan_slots + fa_plan_order with an entry buffer)",
                  NSPLIT, 256 / NSPLIT);
    if (P.plan_maxb > gather_maxb(true, GD * GD))
      return fail(FA_E_ARG, "gather plan chunks hold up to %d blocks, the kernel %d: plan with fa_plan_gather_form",
                  P.plan_maxb, gather_maxb(true, GD * GD));
    if (P.nchunks >= (1ll << 31)) return fail(FA_E_CAPACITY, "gather plan has %lld chunks", (long long)P.nchunks);
  }
  double* rec = nullptr;
  uint32_t* mask = nullptr;
  int rc;
  if (W.mode == GatherStage::FULL) {
    if ((rc = scratch_alloc((void**)&rec, sizeof(double) * R::count(nc), s))) return rc;
    if (bc && (rc = scratch_alloc((void**)&mask, sizeof(uint32_t) * nc, s))) return rc;
  } else {
    rec = reinterpret_cast<double*>(W.work);
    mask = bc ? reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(W.work) + rec_bytes) : nullptr;
  }
  if (nc > 0 && W.mode != GatherStage::ROWS) {
    k_neo_records_m<GD, NN, NQ><<<grid_for((nc + 63) / 64 * 64), 256, 0, s>>>(P.M, P.F, P.tab, bc, rec, mask);
    LAUNCH_CHECK();
  }
  P.rec = rec;
  P.bcmask = mask;
  if (rows) {
    uint32_t* zero32 = nullptr;
    double* dump = nullptr;
    if ((rc = lin_scratch(&zero32, &dump))) return rc;
    int64_t* ldesc = nullptr;
    if ((rc = lin_chunk_desc(P, &ldesc, s, P.corder))) return rc;
    const int64_t grid = gather_grid(k_gather_neo<GD, NN, NQ, NSPLIT>, P.nchunks, 256);
    k_gather_neo<GD, NN, NQ, NSPLIT><<<(unsigned)grid, 256, 0, s>>>(P, zero32, dump, (P.nchunks + 7) / 8);
    LAUNCH_CHECK();
    HIP_TRY(hipFreeAsync(ldesc, s));
    if (bc) {  // Dirichlet diagonals (dolfinx set_diagonal) of the plan's rows
      launch_bc_diag<GD>(P.A, (P.A.row_end - P.A.row_begin) * GD, bc, P.diag, P.err, s);
      LAUNCH_CHECK();
    }
  }
  if (W.mode == GatherStage::FULL) {
    HIP_TRY(hipFreeAsync(rec, s));
    if (mask) HIP_TRY(hipFreeAsync(mask, s));
  }
  return FA_OK;
}

template <int GD, int NN, int NV, int NQ, int NSPLIT, int MAT>
static int launch_gather(GatherArgs P, const int8_t* bc, hipStream_t s, const GatherStage& W) {
  using R = Rec<GD, NV, NQ, MAT>;
  if constexpr (MAT == FA_NEO_HOOKEAN) {
    // the neo-Hookean M gather (k_gather_neo) and its records; its plans must be positional
    static_assert(R::SIMP && NN % NSPLIT == 0 && NN * GD <= 32 && NN < 64, "neo-Hookean gather: simplices");
    return launch_gather_neo<GD, NN, NQ, NSPLIT>(P, bc, s, W);
  } else {
  // ordered (packed) slots are read only by the affine-simplex linear kernel of the same NSPLIT;
  // any other kernel searches its slots in LDS instead
  if (P.slot_order && !((MAT == 0 || MAT == MAT_LINU || MAT == MAT_AFFT) && R::SIMP &&
                        NN % NSPLIT == 0 && P.slot_order == NSPLIT)) {
    P.slots = nullptr;
    P.slot_order = 0;
    P.eadj = nullptr;
  }
  // a positional plan's slot map is by position: a kernel without positional items (k_gather's
  // POSM) cannot read it -- search the slots in LDS instead
  constexpr bool POSM_K = (MAT == 0 || MAT == MAT_LINU || (MAT == MAT_AFFT && NN * GD <= 32)) && R::SIMP &&
                          NN % NSPLIT == 0;
  if (P.eadj && !POSM_K) {
    P.slots = nullptr;
    P.slot_order = 0;
    P.eadj = nullptr;
  }
  static_assert(NN * GD <= 32 || MAT == MAT_AFFT, "bc mask holds 32 dofs");
  if (P.plan_maxb > gather_maxb(false, GD * GD))
    return fail(FA_E_ARG, "gather plan chunks hold up to %d blocks, this form's kernel %d: plan with fa_plan_gather_form",
                P.plan_maxb, gather_maxb(false, GD * GD));
  // the chunk visiting order (fa_plan_locality): k_gather_lin walks it per XCD (lin_chunk_desc);
  // the generic k_gather keeps row order (its static grid measured 50.0 vs 51.5 ms on config E in
  // Morton order, round 2)
  const int32_t* seq = P.corder;
  P.corder = nullptr;
  const int64_t per8 = (P.nchunks + 7) / 8;
  if constexpr (MAT == MAT_LINU && R::SIMP && NN == GD + 1 && NN % NSPLIT == 0 && FA_LIN_FUSE) {
    // P1 simplices through fa_assemble_matrix: k_gather_lin forms the records itself (FUSE)
    constexpr int LNT = lin_threads(GD, NN);
    // Only when the dofmap IS the geometry dofmap: the pack is indexed by vertex id and built over the
    // space's nodes, which are then the vertices (num_nodes == num_vertices). A space with its own P1
    // numbering (FunctionSpace.from_dofmap, a rank's slab) may have more or fewer nodes than the mesh
    // has vertices: it assembles through the records kernel (bc bits read by dof node, cell_bcmask).
    if (W.mode == GatherStage::FULL && P.nchunks > 0 && P.F.E && !P.cw && P.eadj && P.M.geom == P.M.cells &&
        P.slots && P.slot_order == NSPLIT && !P.corder && P.plan_maxadj * NSPLIT <= LNT && P.plan_maxadj >= 0 &&
        P.plan_maxb <= lin_maxb(GD, NN) && P.nchunks < (1ll << 31)) {
      int rc;
      double* xp = nullptr;
      if ((rc = scratch_alloc((void**)&xp, sizeof(double) * 4 * (size_t)std::max<int64_t>(P.M.nnodes, 1), s))) return rc;
      if (P.M.nnodes > 0) {
        k_pack_nodes<GD><<<grid_for(P.M.nnodes), 256, 0, s>>>(P.M.x, bc, P.M.nnodes, xp);
        LAUNCH_CHECK();
      }
      P.xpack = xp;
      P.bcmask = bc ? reinterpret_cast<const uint32_t*>(xp) : nullptr;  // only "has bcs" is read
      P.rec = nullptr;
      const double nu = P.F.nu;
      P.rlm = 2.0 * nu / (1.0 - 2.0 * nu);
      P.trc = 1.0 / (1.0 + P.rlm);
      uint32_t* zero32 = nullptr;
      double* dump = nullptr;
      if ((rc = lin_scratch(&zero32, &dump))) return rc;
      P.fixc = lin_fix_bound(GD, NN, P.rlm, P.trc, P.amax);
      int64_t* ldesc = nullptr;
      if ((rc = lin_chunk_desc(P, &ldesc, s, seq))) return rc;
      if (P.fix) {
        const int64_t grid = gather_grid(k_gather_lin<GD, NN, NSPLIT, LNT, true, true>, P.nchunks, LNT);
        k_gather_lin<GD, NN, NSPLIT, LNT, true, true><<<(unsigned)grid, LNT, 0, s>>>(P, zero32, dump, per8);
      } else {
        const int64_t grid = gather_grid(k_gather_lin<GD, NN, NSPLIT, LNT, true>, P.nchunks, LNT);
        k_gather_lin<GD, NN, NSPLIT, LNT, true><<<(unsigned)grid, LNT, 0, s>>>(P, zero32, dump, per8);
      }
      LAUNCH_CHECK();
      HIP_TRY(hipFreeAsync(ldesc, s));
      if (bc) {
        launch_bc_diag<GD>(P.A, (P.A.row_end - P.A.row_begin) * GD, bc, P.diag, P.err, s);
        LAUNCH_CHECK();
      }
      HIP_TRY(hipFreeAsync(xp, s));
      return FA_OK;
    }
  }
  const int64_t nc = P.M.ncells;
  const int64_t rec_bytes = align256((int64_t)sizeof(double) * R::count(nc));
  if (W.mode == GatherStage::SIZE) {
    *W.bytes = rec_bytes + align256((int64_t)sizeof(uint32_t) * nc);
    return FA_OK;
  }
  double* rec = nullptr;
  uint32_t* mask = nullptr;
  int rc;
  if (W.mode == GatherStage::FULL) {
    if ((rc = scratch_alloc((void**)&rec, sizeof(double) * R::count(nc), s))) return rc;
    if (bc && (rc = scratch_alloc((void**)&mask, sizeof(uint32_t) * nc, s))) return rc;
  } else {
    rec = reinterpret_cast<double*>(W.work);
    mask = bc ? reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(W.work) + rec_bytes) : nullptr;
  }
  if (nc > 0 && W.mode != GatherStage::ROWS) {
    // uniform-nu records of <= 32 dofs: their bc bits from the constrained nodes (k_rec_bcbits), so the
    // records kernel reads no dofmap (config E: records 1.88 -> ~1.5 ms)
    constexpr bool NODE_BITS = (MAT == MAT_LINU || MAT == MAT_AFFT) && NN * GD <= 32 && R::SIZE <= 16;
    const bool node_bits = NODE_BITS && bc && P.adj_ptr && P.adj_idx;
    if constexpr (R::SIZE <= 16)  // small records: stored through LDS as contiguous runs
      k_cell_records_staged<GD, NN, NV, NQ, MAT><<<grid_for(nc), 256, 0, s>>>(P.M, P.F, P.tab, node_bits ? nullptr : bc,
                                                                             rec, mask);
    else k_cell_records<GD, NN, NV, NQ, MAT><<<grid_for(nc), 256, 0, s>>>(P.M, P.F, P.tab, bc, rec, mask);
    LAUNCH_CHECK();
    if constexpr (NODE_BITS) {
      if (node_bits && P.M.nnodes > 0) {
        k_rec_bcbits<GD, NN, R::SIZE><<<grid_for((P.M.nnodes + 7) / 8), 256, 0, s>>>(P.adj_ptr, P.adj_idx, bc, P.M.nnodes,
                                                                                  rec, mask);
        LAUNCH_CHECK();
      }
    }
  }
  P.rec = rec;
  P.bcmask = mask;
  // the store-decoupled gather (k_gather_lin): positional plans of <= 256 items per chunk; affine
  // simplices, and (round 6) affine quadrilaterals / Q1 hexahedra, whose uniform-nu records (s Ji, sign
  // and bc bits) are the simplices' and whose reference tensor packs the same way (get_tables)
  if constexpr ((MAT == MAT_LINU || MAT == MAT_AFFT) && R::SIMP && NN % NSPLIT == 0 && NN * GD <= 32 && NN < 64) {
    constexpr int LNT = lin_threads(GD, NN);
    if (P.nchunks > 0 && W.mode != GatherStage::PREP && !P.cw && P.eadj && P.slots && (NN == GD + 1 || P.pk) &&
        P.slot_order == NSPLIT && !P.corder && P.plan_maxadj * NSPLIT <= LNT && P.plan_maxadj >= 0) {
      if (P.plan_maxb > lin_maxb(GD, NN))
        return fail(FA_E_ARG, "gather plan chunks hold up to %d blocks, the kernel %d", P.plan_maxb, lin_maxb(GD, NN));
      if (P.nchunks >= (1ll << 31)) return fail(FA_E_CAPACITY, "gather plan has %lld chunks", (long long)P.nchunks);
      const double nu = P.F.nu, rr = 2.0 * nu / (1.0 - 2.0 * nu);
      P.trc = 1.0 / (1.0 + rr);
      P.rlm = rr;
      uint32_t* zero32 = nullptr;
      double* dump = nullptr;
      if ((rc = lin_scratch(&zero32, &dump))) return rc;
      P.fixc = lin_fix_bound(GD, NN, rr, P.trc, P.pkmax);  // records scaled by 1 / sqrt(D): |N| bounds
      int64_t* ldesc = nullptr;
      if ((rc = lin_chunk_desc(P, &ldesc, s, seq))) return rc;
      if (P.fix) {
        const int64_t grid = gather_grid(k_gather_lin<GD, NN, NSPLIT, LNT, false, true>, P.nchunks, LNT);
        k_gather_lin<GD, NN, NSPLIT, LNT, false, true><<<(unsigned)grid, LNT, 0, s>>>(P, zero32, dump, per8);
      } else {
        const int64_t grid = gather_grid(k_gather_lin<GD, NN, NSPLIT, LNT>, P.nchunks, LNT);
        k_gather_lin<GD, NN, NSPLIT, LNT><<<(unsigned)grid, LNT, 0, s>>>(P, zero32, dump, per8);
      }
      LAUNCH_CHECK();
      HIP_TRY(hipFreeAsync(ldesc, s));
      if (bc) {  // Dirichlet diagonals (dolfinx set_diagonal) of the plan's rows
        launch_bc_diag<GD>(P.A, (P.A.row_end - P.A.row_begin) * GD, bc, P.diag, P.err, s);
        LAUNCH_CHECK();
      }
      if (W.mode == GatherStage::FULL) {
        HIP_TRY(hipFreeAsync(rec, s));
        if (mask) HIP_TRY(hipFreeAsync(mask, s));
      }
      return FA_OK;
    }
  }
  if (P.nchunks > 0 && W.mode != GatherStage::PREP) {
    if (P.fix)
      return fail(FA_E_UNSUPPORTED, "deterministic assembly runs the affine-simplex elasticity gather (uniform nu, "
                                    "positional plan: fa_plan_slots + fa_plan_order with an entry buffer) only");
    int64_t* desc = nullptr;
    if ((rc = chunk_desc(P, &desc, s))) return rc;
    const int64_t grid = gather_grid(k_gather<GD, NN, NV, NQ, NSPLIT, MAT>, P.nchunks);
    double* bhat = nullptr;
    if constexpr (MAT == MAT_AFFT) {  // the kernel forms B_ab = r Ahat_ab + Ahat_ab^T per block
      const double nu = P.F.nu;
      P.rlm = 2.0 * nu / (1.0 - 2.0 * nu);
      P.trc = 1.0 / (1.0 + P.rlm);
    }
    if constexpr (MAT == MAT_LINU) {  // B_ab = r Ahat_ab + Ahat_ab^T for this form's nu
      const double nu = P.F.nu, rr = 2.0 * nu / (1.0 - 2.0 * nu);
      if ((rc = scratch_alloc((void**)&bhat, sizeof(double) * NN * NN * GD * GD, s))) return rc;
      k_bhat<GD><<<grid_for(NN * NN), 256, 0, s>>>(P.ahat, NN * NN, rr, bhat);
      LAUNCH_CHECK();
      P.ahat = bhat;
      P.trc = 1.0 / (1.0 + rr);
      P.rlm = rr;
    }
    bool launched = false;
    if constexpr (MAT == MAT_LINU && Rec<GD, NV, NQ, MAT>::SIMP && NN * GD <= 32 && NN * NN < 127) {
      if (P.cw) {  // contribution plan: the block-owner gather
        if (P.plan_maxb > own_maxb(GD * GD))
          return fail(FA_E_ARG, "contribution plan chunks hold %d blocks, the kernel %d", P.plan_maxb, own_maxb(GD * GD));
        const int64_t go = gather_grid(k_gather_own<GD, NN>, P.nchunks);
        k_gather_own<GD, NN><<<(unsigned)go, 256, 0, s>>>(P);
        launched = true;
      }
    }
    if (!launched) k_gather<GD, NN, NV, NQ, NSPLIT, MAT><<<(unsigned)grid, 256, 0, s>>>(P);
    LAUNCH_CHECK();
    HIP_TRY(hipFreeAsync(desc, s));
    if (bhat) HIP_TRY(hipFreeAsync(bhat, s));
  }
  if (W.mode == GatherStage::FULL) {
    HIP_TRY(hipFreeAsync(rec, s));
    if (mask) HIP_TRY(hipFreeAsync(mask, s));
  }
  return FA_OK;
  }
}

// Hexahedra: MFMA element blocks into a stream-ordered block store, then the row gather sums
// them (the "store pass + per-destination sum pass" alternative to global atomics).
template <int NN, int NQ, int NSPLIT>
static int launch_hex_gather(GatherArgs P, const DevTables& T, const int8_t* bc, hipStream_t s, const GatherStage& W) {
  const int64_t nc = P.M.ncells;
  if (P.slot_order) {
    P.slots = nullptr;
    P.slot_order = 0;
    P.eadj = nullptr;
  }
  if (W.mode == GatherStage::SIZE) {
    *W.bytes = align256((int64_t)sizeof(double) * 9 * NN * NN * nc);
    return FA_OK;
  }
  double* eb = nullptr;
  int rc;
  if (W.mode == GatherStage::FULL) {
    if ((rc = scratch_alloc((void**)&eb, sizeof(double) * 9 * NN * NN * nc, s))) return rc;
  } else {
    eb = reinterpret_cast<double*>(W.work);
  }
  if (nc > 0 && W.mode != GatherStage::ROWS) {
    constexpr int thr = hex_threads_m(NN, 2);
    // one workgroup per cell (a resident grid looping over the cells with the next cell's inputs
    // prefetched measured 41.7 vs 41.5 ms on config Dmfma, round 5)
    const int grid = (int)std::min<int64_t>(nc, kMaxBlocks);
    BsrView none{nullptr, nullptr, nullptr, 0, 0};
    k_hex_mfma<NN, NQ, 2><<<grid, thr, 0, s>>>(P.M, P.F, T, 0, nc, eb, none, bc, P.err);
    LAUNCH_CHECK();
  }
  P.rec = eb;
  P.bcmask = nullptr;
  if (P.nchunks > 0 && W.mode != GatherStage::PREP) {
    if (P.fix) return fail(FA_E_UNSUPPORTED, "deterministic assembly: not for non-affine hexahedra");
    int64_t* desc = nullptr;
    if ((rc = chunk_desc(P, &desc, s))) return rc;
    const int64_t grid = gather_grid(k_gather<3, NN, 8, NQ, NSPLIT, MAT_BLOCKS>, P.nchunks);
    k_gather<3, NN, 8, NQ, NSPLIT, MAT_BLOCKS><<<(unsigned)grid, 256, 0, s>>>(P);
    LAUNCH_CHECK();
    HIP_TRY(hipFreeAsync(desc, s));
  }
  if (W.mode == GatherStage::FULL) HIP_TRY(hipFreeAsync(eb, s));
  return FA_OK;
}

// the uniform-nu affine-simplex kernels (MAT_LINU): E per cell with one nu, away from nu = 1/2
static bool lin_uniform_nu(const FormView& F) {
  return F.kind == FA_LINEAR_ELASTICITY && F.E && F.nu > -0.99 && F.nu < 0.49;
}

static int dispatch_gather(const fa_mesh* m, const DevTables& T, int kind, const GatherArgs& P, const int8_t* bc,
                           hipStream_t s, bool* handled, const GatherStage& W = GatherStage()) {
  *handled = true;
  if (m->cell_type == FA_HEXAHEDRON && kind == FA_LINEAR_ELASTICITY && P.affine && lin_uniform_nu(P.F)) {
    // affine hexahedra: the row gather computes every block from the cell's Jacobian and the 1-D
    // matrices (MAT_AFFT); the MFMA element kernel + block store serves general trilinear cells
    if (m->degree == 1 && T.nq == 8) return launch_gather<3, 8, 8, 8, 2, MAT_AFFT>(P, bc, s, W);
    if (m->degree == 2 && T.nq == 27) return launch_gather<3, 27, 8, 27, FA_Q2HEX_NSPLIT, MAT_AFFT>(P, bc, s, W);
    if (m->degree == 3 && T.nq == 64) return launch_gather<3, 64, 8, 64, FA_Q3HEX_NSPLIT, MAT_AFFT>(P, bc, s, W);
  }
  if (m->cell_type == FA_QUADRILATERAL && kind == FA_LINEAR_ELASTICITY && P.affine && lin_uniform_nu(P.F)) {
    if (m->degree == 1 && T.nq == 4) return launch_gather<2, 4, 4, 4, 1, MAT_AFFT>(P, bc, s, W);
    if (m->degree == 2 && T.nq == 9) return launch_gather<2, 9, 4, 9, FA_Q2QUAD_NSPLIT, MAT_AFFT>(P, bc, s, W);
    if (m->degree == 3 && T.nq == 16) return launch_gather<2, 16, 4, 16, 4, MAT_AFFT>(P, bc, s, W);
  }
  if (m->cell_type == FA_HEXAHEDRON && kind == FA_LINEAR_ELASTICITY) {
    if (m->degree == 1 && T.nq == 8) return launch_hex_gather<8, 8, 1>(P, T, bc, s, W);
    if (m->degree == 2 && T.nq == 27) return launch_hex_gather<27, 27, 3>(P, T, bc, s, W);
    if (m->degree == 3 && T.nq == 64) return launch_hex_gather<64, 64, 8>(P, T, bc, s, W);
  }
  const int ct = m->cell_type, p = m->degree, nq = T.nq;
  if (kind == FA_ASYM_DAMAGE) return launch_gather<2, 3, 3, 1, 1, FA_ASYM_DAMAGE>(P, bc, s, W);
  if (kind == FA_NEO_HOOKEAN) {
    if (ct == FA_TETRAHEDRON && p == 2 && nq == 4) return launch_gather<3, 10, 4, 4, FA_NEO_NSPLIT, FA_NEO_HOOKEAN>(P, bc, s, W);
    // P1 tets: the column split of the plan's order (lin_simplex_nsplit), so the positional slot map fits
    if (ct == FA_TETRAHEDRON && p == 1 && nq == 1) return launch_gather<3, 4, 4, 1, FA_P1TET_NSPLIT, FA_NEO_HOOKEAN>(P, bc, s, W);
    if (ct == FA_TRIANGLE && p == 2 && nq == 3) return launch_gather<2, 6, 3, 3, 2, FA_NEO_HOOKEAN>(P, bc, s, W);
    if (ct == FA_TRIANGLE && p == 1 && nq == 1) return launch_gather<2, 3, 3, 1, 1, FA_NEO_HOOKEAN>(P, bc, s, W);
    *handled = false;
    return FA_OK;
  }
  if (lin_uniform_nu(P.F)) {
    if (ct == FA_TRIANGLE && p == 1 && nq == 1) return launch_gather<2, 3, 3, 1, 1, MAT_LINU>(P, bc, s, W);
    if (ct == FA_TRIANGLE && p == 2 && nq == 3) return launch_gather<2, 6, 3, 3, 2, MAT_LINU>(P, bc, s, W);
    if (ct == FA_TETRAHEDRON && p == 1 && nq == 1) return launch_gather<3, 4, 4, 1, FA_P1TET_NSPLIT, MAT_LINU>(P, bc, s, W);
    if (ct == FA_TETRAHEDRON && p == 2 && nq == 4)
      return launch_gather<3, 10, 4, 4, FA_P2TET_NSPLIT, MAT_LINU>(P, bc, s, W);
  }
  if (ct == FA_TRIANGLE && p == 1 && nq == 1) return launch_gather<2, 3, 3, 1, 1, 0>(P, bc, s, W);
  if (ct == FA_TRIANGLE && p == 2 && nq == 3) return launch_gather<2, 6, 3, 3, 2, 0>(P, bc, s, W);
  // the column split of the plan's order (lin_simplex_nsplit): a P1-tet plan ordered for
  // FA_P1TET_NSPLIT keeps its positional slot map with this kernel too
  if (ct == FA_TETRAHEDRON && p == 1 && nq == 1) return launch_gather<3, 4, 4, 1, FA_P1TET_NSPLIT, 0>(P, bc, s, W);
  if (ct == FA_TETRAHEDRON && p == 2 && nq == 4) return launch_gather<3, 10, 4, 4, FA_P2TET_NSPLIT, 0>(P, bc, s, W);
  if (ct == FA_QUADRILATERAL && p == 1 && nq == 4) return launch_gather<2, 4, 4, 4, 1, 0>(P, bc, s, W);
  if (ct == FA_QUADRILATERAL && p == 2 && nq == 9) return launch_gather<2, 9, 4, 9, 3, 0>(P, bc, s, W);
  *handled = false;
  return FA_OK;
}

static int launch_cell_blocks(int mode, const fa_mesh* mesh, const MeshView& M, const FormView& F, const DevTables& T,
                              int64_t c0, int64_t nc, double* Ae, const BsrView& A, const int8_t* bc, int* derr,
                              hipStream_t s) {
  int64_t total = nc * (int64_t)T.nn * T.nn;
  if (total <= 0) return FA_OK;
  int grid = grid_for(total);
#define CB(GD, NV)                                                                                             \
  do {                                                                                                         \
    if (mode == 0) k_cell_blocks<GD, NV, 0><<<grid, 256, 0, s>>>(M, F, T, c0, nc, Ae, A, bc, derr);             \
    else k_cell_blocks<GD, NV, 1><<<grid, 256, 0, s>>>(M, F, T, c0, nc, Ae, A, bc, derr);                      \
  } while (0)
  switch (mesh->cell_type) {
    case FA_TRIANGLE: CB(2, 3); break;
    case FA_QUADRILATERAL: CB(2, 4); break;
    case FA_TETRAHEDRON: CB(3, 4); break;
    case FA_HEXAHEDRON: CB(3, 8); break;
    default: return fail(FA_E_UNSUPPORTED, "cell type %d", mesh->cell_type);
  }
#undef CB
  LAUNCH_CHECK();
  return FA_OK;
}

extern "C" int fa_tabulate_cells(const fa_mesh* mesh, const fa_form* form, int64_t c0, int64_t ncells_out, double* Ae,
                                 void* stream) {
  int rc = check_mesh(mesh);
  if (rc) return rc;
  if (!Ae && ncells_out > 0) return fail(FA_E_ARG, "null Ae");
  if (c0 < 0 || c0 + ncells_out > mesh->ncells) return fail(FA_E_ARG, "cell range out of bounds");
  FormView F;
  if ((rc = form_view(mesh, form, F))) return rc;
  DevTables T;
  if ((rc = get_tables(mesh->cell_type, mesh->degree, form->qdeg, &T))) return rc;
  MeshView M{mesh->cells, mesh->geom, mesh->x, mesh->ncells, mesh->nnodes, mesh->nn, mesh->nv, mesh->gdim};
  BsrView A{nullptr, nullptr, nullptr, 0, 0};
  bool hex = false;
  rc = launch_hex_mfma(0, mesh, M, F, T, c0, ncells_out, Ae, A, nullptr, nullptr, (hipStream_t)stream, &hex);
  if (rc || hex) return rc;
  return launch_cell_blocks(0, mesh, M, F, T, c0, ncells_out, Ae, A, nullptr, nullptr, (hipStream_t)stream);
}

// Error flags raised by kernels (a pattern entry or diagonal the mesh needs is missing) are read
// back only with FA_CHECK_ERRORS, which synchronises the stream; the timed path stays asynchronous.
extern "C" int fa_assemble_matrix(const fa_mesh* mesh, const fa_form* form, const fa_adjacency* adj, const fa_plan* plan,
                                  const int8_t* bc, double diag, fa_bsr* A, int32_t flags, void* stream) {
  int rc = check_mesh(mesh);
  if (rc) return rc;
  if (!A || !A->indptr || !A->indices || !A->data) return fail(FA_E_ARG, "null matrix");
  if (A->bs != mesh->gdim || A->nrows != mesh->nnodes) return fail(FA_E_ARG, "matrix shape does not match mesh");
  int64_t wb = A->row_begin, we = A->row_end;
  if (we <= wb) { wb = 0; we = mesh->nnodes; }
  if (wb < 0 || we > mesh->nnodes) return fail(FA_E_ARG, "row window out of range");
  FormView F;
  if ((rc = form_view(mesh, form, F))) return rc;
  DevTables T;
  if ((rc = get_tables(mesh->cell_type, mesh->degree, form->qdeg, &T))) return rc;
  hipStream_t s = (hipStream_t)stream;
  // FA_CHECK_ERRORS: the pattern and adjacency are validated on the device first (fa_check_pattern
  // without its exactness bit: a superset pattern assembles correctly)
  if ((flags & FA_CHECK_ERRORS) && adj && adj->ptr && adj->idx &&
      (rc = check_pattern(mesh, adj, A->indptr, A->indices, A->nblocks, false, stream)))
    return rc;
  MeshView M{mesh->cells, mesh->geom, mesh->x, mesh->ncells, mesh->nnodes, mesh->nn, mesh->nv, mesh->gdim};
  BsrView Av{A->indptr, A->indices, A->data, wb, we};
  static int* derr = nullptr;  // per-process device error word (sticky until read)
  if (!derr) {
    HIP_TRY(hipMalloc((void**)&derr, sizeof(int)));
    HIP_TRY(hipMemset(derr, 0, sizeof(int)));
  }
  bool scatter = (flags & FA_SCATTER) != 0;
  if (!scatter) {
    if (!adj || !adj->ptr || !adj->idx || !plan || !plan->row_start)
      return fail(FA_E_ARG, "FA_GATHER needs the adjacency and a plan (fa_plan_gather)");
    GatherArgs P{};
    P.M = M; P.F = F; P.A = Av;
    P.adj_ptr = adj->ptr; P.adj_idx = adj->idx; P.row_start = plan->row_start; P.nchunks = plan->nchunks; P.corder = plan->corder; P.chunk_desc = plan->chunk_desc; P.plan_maxb = plan->max_blocks; P.plan_maxadj = plan->max_adj;
    P.slots = plan->slots;
    P.slot_order = plan->slots ? plan->slot_order : 0;
    P.eadj = P.slot_order ? plan->eadj : nullptr;
    P.bc = bc; P.diag = diag; P.tab = T.wq; P.ahat = T.ahat; P.rec = nullptr; P.bcmask = nullptr; P.err = derr; P.xpack = nullptr;
    P.affine = (plan->cell_flags & FA_PLAN_AFFINE) != 0;
    P.t1d = T.t1d; P.lat = T.lat;
    P.fix = ((flags & FA_DETERMINISTIC) || (plan->cell_flags & FA_PLAN_DETERMINISTIC)) ? 1 : 0;
    P.amax = T.amax;
    P.pk = T.pk; P.pks = T.pk_scale; P.pkmax = T.pk_amax;
    set_contrib(P, plan);
    if (P.fix && P.cw) return fail(FA_E_UNSUPPORTED, "deterministic assembly: not with a contribution plan");
    bool handled = false;
    rc = dispatch_gather(mesh, T, F.kind, P, bc, s, &handled);
    if (rc) return rc;
    if (!handled && P.fix) return fail(FA_E_UNSUPPORTED, "deterministic assembly: no gather kernel for this form");
    if (!handled) scatter = true;  // no specialised gather kernel: generic element scatter
  }
  if (scatter) {
    // the generic fallback of FA_GATHER writes every value, so it starts from zero;
    // FA_SCATTER accumulates into A unless FA_ZERO_FIRST (MatZeroEntries) is set
    if (!(flags & FA_SCATTER) || (flags & FA_ZERO_FIRST))
    {
      k_zero_window<<<4096, 256, 0, s>>>(Av, A->bs * A->bs);
      LAUNCH_CHECK();
    }
    bool hex = false;
    rc = launch_hex_mfma(1, mesh, M, F, T, 0, mesh->ncells, nullptr, Av, bc, derr, s, &hex);
    if (rc) return rc;
    if (!hex) rc = launch_cell_blocks(1, mesh, M, F, T, 0, mesh->ncells, nullptr, Av, bc, derr, s);
    if (rc) return rc;
    if (bc) {
      int64_t n = (we - wb) * mesh->gdim;
      if (mesh->gdim == 2) launch_bc_diag<2>(Av, n, bc, diag, derr, s);
      else launch_bc_diag<3>(Av, n, bc, diag, derr, s);
      LAUNCH_CHECK();
    }
  }
  if (flags & FA_CHECK_ERRORS) {
    int herr = 0;
    HIP_TRY(hipMemcpyAsync(&herr, derr, sizeof(int), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    if (herr) {
      HIP_TRY(hipMemset(derr, 0, sizeof(int)));
      return fail(FA_E_PATTERN, "assembly kernel flagged error 0x%x (missing pattern entry / diagonal)", herr);
    }
  }
  return FA_OK;
}

// ------------------------------------------------------------------------------------ split gather
// fa_assemble_matrix(FA_GATHER) in two calls on a caller-owned work buffer, so that a caller can
// assemble some rows (a rank's interface planes), start their exchange, and assemble the rest
// while it runs -- without recomputing the per-cell records (femasm.parallel).
static int gather_stage(const fa_mesh* mesh, const fa_form* form, const fa_adjacency* adj, const fa_plan* plan,
                        const int8_t* bc, double diag, const fa_bsr* A, const GatherStage& W, hipStream_t s) {
  int rc = check_mesh(mesh);
  if (rc) return rc;
  FormView F;
  if ((rc = form_view(mesh, form, F))) return rc;
  DevTables T;
  if ((rc = get_tables(mesh->cell_type, mesh->degree, form->qdeg, &T))) return rc;
  MeshView M{mesh->cells, mesh->geom, mesh->x, mesh->ncells, mesh->nnodes, mesh->nn, mesh->nv, mesh->gdim};
  GatherArgs P{};
  P.M = M; P.F = F;
  P.A = BsrView{nullptr, nullptr, nullptr, 0, 0};
  P.tab = T.wq; P.ahat = T.ahat; P.bc = bc; P.diag = diag;
  P.affine = 0;  // the prepare stage has no plan: tensor cells keep the element-kernel path
  P.t1d = T.t1d; P.lat = T.lat;
  static int* derr = nullptr;  // device error word of the split path
  if (!derr) {
    HIP_TRY(hipMalloc((void**)&derr, sizeof(int)));
    HIP_TRY(hipMemset(derr, 0, sizeof(int)));
  }
  P.err = derr;
  if (adj && adj->ptr && adj->idx) {  // (the prepare stage: the records' bc bits from the nodes, k_rec_bcbits)
    P.adj_ptr = adj->ptr;
    P.adj_idx = adj->idx;
  }
  if (W.mode == GatherStage::ROWS) {
    if (!A || !A->indptr || !A->indices || !A->data) return fail(FA_E_ARG, "null matrix");
    if (A->bs != mesh->gdim || A->nrows != mesh->nnodes) return fail(FA_E_ARG, "matrix shape does not match mesh");
    int64_t wb = A->row_begin, we = A->row_end;
    if (we <= wb) { wb = 0; we = mesh->nnodes; }
    if (wb < 0 || we > mesh->nnodes) return fail(FA_E_ARG, "row window out of range");
    if (!adj || !adj->ptr || !adj->idx || !plan || !plan->row_start)
      return fail(FA_E_ARG, "fa_gather_rows needs the adjacency and a plan (fa_plan_gather)");
    P.A = BsrView{A->indptr, A->indices, A->data, wb, we};
    P.adj_ptr = adj->ptr; P.adj_idx = adj->idx; P.row_start = plan->row_start; P.nchunks = plan->nchunks; P.corder = plan->corder; P.chunk_desc = plan->chunk_desc; P.plan_maxb = plan->max_blocks; P.plan_maxadj = plan->max_adj;
    P.slots = plan->slots;
    P.slot_order = plan->slots ? plan->slot_order : 0;
    P.eadj = P.slot_order ? plan->eadj : nullptr;
    P.fix = (plan->cell_flags & FA_PLAN_DETERMINISTIC) ? 1 : 0;
    P.amax = T.amax;
    P.pk = T.pk; P.pks = T.pk_scale; P.pkmax = T.pk_amax;
    set_contrib(P, plan);
    if (P.fix && P.cw) return fail(FA_E_UNSUPPORTED, "deterministic assembly: not with a contribution plan");
  }
  bool handled = false;
  rc = dispatch_gather(mesh, T, F.kind, P, bc, s, &handled, W);
  if (rc) return rc;
  if (!handled) return fail(FA_E_UNSUPPORTED, "no gather kernel for this element/form: use fa_assemble_matrix");
  return FA_OK;
}

extern "C" int fa_gather_work_bytes(const fa_mesh* mesh, const fa_form* form, int64_t* bytes) {
  if (!bytes) return fail(FA_E_ARG, "null bytes");
  GatherStage W;
  W.mode = GatherStage::SIZE;
  W.bytes = bytes;
  return gather_stage(mesh, form, nullptr, nullptr, nullptr, 0.0, nullptr, W, nullptr);
}

extern "C" int fa_gather_prepare(const fa_mesh* mesh, const fa_form* form, const int8_t* bc, void* work,
                                 void* stream) {
  if (!work) return fail(FA_E_ARG, "null work buffer");
  GatherStage W;
  W.mode = GatherStage::PREP;
  W.work = work;
  return gather_stage(mesh, form, nullptr, nullptr, bc, 0.0, nullptr, W, (hipStream_t)stream);
}

extern "C" int fa_gather_rows(const fa_mesh* mesh, const fa_form* form, const fa_adjacency* adj, const fa_plan* plan,
                              const int8_t* bc, double diag, const void* work, fa_bsr* A, void* stream) {
  if (!work) return fail(FA_E_ARG, "null work buffer");
  GatherStage W;
  W.mode = GatherStage::ROWS;
  W.work = const_cast<void*>(work);
  return gather_stage(mesh, form, adj, plan, bc, diag, A, W, (hipStream_t)stream);
}

// ------------------------------------------------------------------------------------ vectors (next rows)
// Damage-law stress at the single quadrature point, multiplied by w: restated from asym_stress
// (hand version, MFEM/mechanic2d/asym_elasto_damage_model.cc:207-329). strain = (e00, e11, e01).
__device__ __forceinline__ void damage_stress(double s00, double s11, double s01, double l, double m, double d,
                                              double w, double (&sig)[2][2]) {
  const double limit = 1.e-12, mlimit = -1.e-12;
  sig[0][0] = sig[0][1] = sig[1][0] = sig[1][1] = 0.0;
  if (d > 0.0) {
    double I1 = s00 + s11, I2 = s01 * s01 - s00 * s11;
    if (I1 > limit || I2 > limit || I1 < mlimit || I2 < mlimit) {
      double delta = I1 * I1 + 4.0 * I2;
      double r = sqrt(fmax(0.0, delta));
      double ev0 = 0.5 * (I1 + r), ev1 = 0.5 * (I1 - r);
      double a1 = ev0 >= 0.0 ? 1.0 : 0.0, a2 = ev1 >= 0.0 ? 1.0 : 0.0, a = (ev0 + ev1) >= 0.0 ? 1.0 : 0.0;
      if (!((d == 1.0) && (a == 1.0) && (a1 == 1.0) && (a2 == 1.0))) {
        double V00, V01, V10, V11;
        if (fabs(s01) > limit) {
          V00 = ev0 - s11; V01 = ev1 - s11; V10 = V11 = s01;
          double n0 = sqrt(V00 * V00 + V10 * V10), n1 = sqrt(V01 * V01 + V11 * V11);
          V00 /= n0; V10 /= n0; V01 /= n1; V11 /= n1;
        } else {
          V00 = V11 = 1.0; V10 = V01 = 0.0;
        }
        double temp = 2.0 * m * w, gam = 0.5 * l / m;
        double c = 1.0 - a * d, c1 = 1.0 - a1 * d, c2 = 1.0 - a2 * d;
        double D0 = temp * (c1 + gam * c), D1 = temp * gam * c, D2 = temp * (c2 + gam * c);
        double e0 = D0 * ev0 + D1 * ev1, e1 = D1 * ev0 + D2 * ev1;
        sig[0][0] = V00 * e0 * V00 + V01 * e1 * V01;
        sig[1][1] = V10 * e0 * V10 + V11 * e1 * V11;
        sig[0][1] = sig[1][0] = V00 * e0 * V10 + V01 * e1 * V11;
      }
    }
  } else {
    double m2plw = w * (2.0 * m + l), lw = l * w;
    sig[0][0] = m2plw * s00 + lw * s11;
    sig[1][1] = m2plw * s11 + lw * s00;
    sig[0][1] = sig[1][0] = w * m * (s01 + s01);
  }
}

// Residual b[a] += sum over the cells of node a of int sigma(u):eps(phi_a e_i) - f.phi_a e_i.
// One thread per node (node-parallel gather through the adjacency): deterministic, one write per dof.
// Ts: tables of the sigma term's rule (the form's degree; the reference's `dxx`), Tf: the load
// term's rule (degree 2p; the reference's default `dx`).
template <int GD, int NV, int MAT>
__global__ __launch_bounds__(256) void k_vector(MeshView M, FormView F, DevTables Ts, DevTables Tf,
                                                const int64_t* __restrict__ adj_ptr,
                                                const int32_t* __restrict__ adj_idx, double* __restrict__ b) {
  const int nn = M.nn;
  for (int64_t a = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; a < M.nnodes; a += (int64_t)gridDim.x * blockDim.x) {
    double r[GD];
#pragma unroll
    for (int i = 0; i < GD; ++i) r[i] = 0.0;
    for (int64_t j = adj_ptr[a]; j < adj_ptr[a + 1]; ++j) {
      const int32_t p = adj_idx[j];
      const int64_t c = p / nn;
      const int aloc = p % nn;
      const int32_t* cn = M.cells + c * nn;
      if (F.u) {
        if constexpr (MAT == FA_ASYM_DAMAGE) {
          double g[3][2], w, H[3][3];
          damage_cell(M, F, c, g, w, H);  // gradients + weight (H unused here)
          double lam, mu;
          cell_lame(F, c, lam, mu);
          double gr[2][2] = {{0.0, 0.0}, {0.0, 0.0}}, dq = 0.0;
          for (int bb = 0; bb < 3; ++bb) {
            int64_t n = cn[bb];
            double u0 = F.u[n * 2], u1 = F.u[n * 2 + 1];
            gr[0][0] += u0 * g[bb][0]; gr[0][1] += u0 * g[bb][1];
            gr[1][0] += u1 * g[bb][0]; gr[1][1] += u1 * g[bb][1];
            if (F.d) dq += F.d[n];
          }
          double sig[2][2];
          if (F.ad) damage_stress_ad(gr[0][0], gr[1][1], 0.5 * (gr[0][1] + gr[1][0]), lam, mu, dq * (1.0 / 3.0), w, sig);
          else damage_stress(gr[0][0], gr[1][1], 0.5 * (gr[0][1] + gr[1][0]), lam, mu, dq * (1.0 / 3.0), w, sig);
#pragma unroll
          for (int i = 0; i < 2; ++i) r[i] += sig[i][0] * g[aloc][0] + sig[i][1] * g[aloc][1];
        } else {
          double lam, mu;
          cell_lame(F, c, lam, mu);
          for (int q = 0; q < Ts.nq; ++q) {
            double Ji[GD][GD];
            const double wd = Ts.wq[q] * cell_geometry_q<GD, NV>(M, c, Ts.gdphi + (size_t)q * NV * GD, Ji);
            double gu[GD][GD];
#pragma unroll
            for (int i = 0; i < GD; ++i)
#pragma unroll
              for (int k = 0; k < GD; ++k) gu[i][k] = 0.0;
            double ga[GD];
            for (int bb = 0; bb < nn; ++bb) {
              double gb[GD];
              phys_grad<GD>(Ts.dphi + ((size_t)q * nn + bb) * GD, Ji, gb);
              if (bb == aloc)
#pragma unroll
                for (int k = 0; k < GD; ++k) ga[k] = gb[k];
              const int64_t n = cn[bb];
#pragma unroll
              for (int i = 0; i < GD; ++i) {
                const double ui = F.u[n * GD + i];
#pragma unroll
                for (int k = 0; k < GD; ++k) gu[i][k] += ui * gb[k];
              }
            }
            if (F.kind == FA_NEO_HOOKEAN) {  // r_a,i += w P_iK(I + grad u) g_a[K]
              double Fq[GD * GD], P[GD * GD];
#pragma unroll
              for (int i = 0; i < GD; ++i)
#pragma unroll
                for (int k = 0; k < GD; ++k) Fq[i * GD + k] = gu[i][k] + (i == k ? 1.0 : 0.0);
              neo_stress_ad<GD>(Fq, lam, mu, P);
#pragma unroll
              for (int i = 0; i < GD; ++i) {
                double s = 0.0;
#pragma unroll
                for (int k = 0; k < GD; ++k) s += P[i * GD + k] * ga[k];
                r[i] += wd * s;
              }
              continue;
            }
            double tr = 0.0;
#pragma unroll
            for (int i = 0; i < GD; ++i) tr += gu[i][i];
#pragma unroll
            for (int i = 0; i < GD; ++i) {
              double s = 0.0;
#pragma unroll
              for (int k = 0; k < GD; ++k) {
                const double sig = mu * (gu[i][k] + gu[k][i]) + (i == k ? lam * tr : 0.0);
                s += sig * ga[k];
              }
              r[i] += wd * s;
            }
          }
        }
      }
      if (F.f) {
        for (int q = 0; q < Tf.nq; ++q) {
          double Ji[GD][GD];
          const double wd = Tf.wq[q] * cell_geometry_q<GD, NV>(M, c, Tf.gdphi + (size_t)q * NV * GD, Ji);
          double fq[GD];
#pragma unroll
          for (int i = 0; i < GD; ++i) fq[i] = 0.0;
          for (int bb = 0; bb < nn; ++bb) {
            const double ph = Tf.phi[(size_t)q * nn + bb];
            const int64_t n = cn[bb];
#pragma unroll
            for (int i = 0; i < GD; ++i) fq[i] += F.f[n * GD + i] * ph;
          }
          const double pa = Tf.phi[(size_t)q * nn + aloc] * wd;
#pragma unroll
          for (int i = 0; i < GD; ++i) r[i] -= fq[i] * pa;
        }
      }
    }
    double o[GD];
#pragma unroll
    for (int i = 0; i < GD; ++i) o[i] = b[a * GD + i] + r[i];
#pragma unroll
    for (int i = 0; i < GD; ++i) b[a * GD + i] = o[i];
    store_fence(o);  // the grid-stride loop's next node would rewrite the store's data registers
  }
}

// dolfinx apply_lifting with one J form: b[a] -= alpha * sum over the cells of a that hold bc dofs
// of K_e[a, j] (g_j - x0_j) for constrained dofs j (element matrices, as dolfinx does per cell).
template <int GD, int NV, int MAT>
__global__ __launch_bounds__(256) void k_lifting(MeshView M, FormView F, DevTables T, const int64_t* __restrict__ adj_ptr,
                                                 const int32_t* __restrict__ adj_idx, const int8_t* __restrict__ bc,
                                                 const double* __restrict__ g, const double* __restrict__ x0,
                                                 double alpha, double* __restrict__ b) {
  const int nn = M.nn;
  for (int64_t a = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; a < M.nnodes; a += (int64_t)gridDim.x * blockDim.x) {
    double r[GD];
#pragma unroll
    for (int i = 0; i < GD; ++i) r[i] = 0.0;
    for (int64_t j = adj_ptr[a]; j < adj_ptr[a + 1]; ++j) {
      const int32_t p = adj_idx[j];
      const int64_t c = p / nn;
      const int aloc = p % nn;
      const int32_t* cn = M.cells + c * nn;
      bool any = false;
      for (int bb = 0; bb < nn && !any; ++bb)
#pragma unroll
        for (int k = 0; k < GD; ++k) any |= bc[(int64_t)cn[bb] * GD + k] != 0;
      if (!any) continue;
      for (int bb = 0; bb < nn; ++bb) {
        const int64_t nb = cn[bb];
        bool hit = false;
#pragma unroll
        for (int k = 0; k < GD; ++k) hit |= bc[nb * GD + k] != 0;
        if (!hit) continue;
        double K[GD][GD];
        if constexpr (MAT == FA_ASYM_DAMAGE) {
          if constexpr (GD == 2) {
            double gg[3][2], w, H[3][3];
            damage_cell(M, F, c, gg, w, H);
            double ga[2] = {gg[aloc][0], gg[aloc][1]}, gb[2] = {gg[bb][0], gg[bb][1]};
            damage_block(ga, gb, w, H, K);
          }
        } else if (F.kind == FA_NEO_HOOKEAN) {  // K_ab of the tangent at the state u
          double lam, mu;
          cell_lame(F, c, lam, mu);
#pragma unroll
          for (int i = 0; i < GD; ++i)
#pragma unroll
            for (int k = 0; k < GD; ++k) K[i][k] = 0.0;
          for (int q = 0; q < T.nq; ++q) {
            double Ji[GD][GD];
            const double wd = T.wq[q] * cell_geometry_q<GD, NV>(M, c, T.gdphi + (size_t)q * NV * GD, Ji);
            double Fq[GD * GD], A[GD * GD * GD * GD];
            deformation_gradient<GD>(F.u, cn, nn, T.dphi + (size_t)q * nn * GD, Ji, Fq);
            neo_tangent_ad<GD>(Fq, lam, mu, A);
            double ga[GD], gb[GD];
            phys_grad<GD>(T.dphi + ((size_t)q * nn + aloc) * GD, Ji, ga);
            phys_grad<GD>(T.dphi + ((size_t)q * nn + bb) * GD, Ji, gb);
            neo_block_add<GD>(A, ga, gb, wd, K);
          }
        } else {
          double lam, mu;
          cell_lame(F, c, lam, mu);
          double G[GD][GD];
#pragma unroll
          for (int i = 0; i < GD; ++i)
#pragma unroll
            for (int k = 0; k < GD; ++k) G[i][k] = 0.0;
          for (int q = 0; q < T.nq; ++q) {
            double Ji[GD][GD];
            const double wd = T.wq[q] * cell_geometry_q<GD, NV>(M, c, T.gdphi + (size_t)q * NV * GD, Ji);
            double ga[GD], gb[GD];
            phys_grad<GD>(T.dphi + ((size_t)q * nn + aloc) * GD, Ji, ga);
            phys_grad<GD>(T.dphi + ((size_t)q * nn + bb) * GD, Ji, gb);
#pragma unroll
            for (int i = 0; i < GD; ++i)
#pragma unroll
              for (int k = 0; k < GD; ++k) G[i][k] += wd * ga[i] * gb[k];
          }
          lin_block<GD>(G, lam, mu, K);
        }
#pragma unroll
        for (int k = 0; k < GD; ++k) {
          if (!bc[nb * GD + k]) continue;
          const double v = g[nb * GD + k] - (x0 ? x0[nb * GD + k] : 0.0);
#pragma unroll
          for (int i = 0; i < GD; ++i) r[i] += K[i][k] * v;
        }
      }
    }
    double o[GD];
#pragma unroll
    for (int i = 0; i < GD; ++i) o[i] = b[a * GD + i] - alpha * r[i];
#pragma unroll
    for (int i = 0; i < GD; ++i) b[a * GD + i] = o[i];
    store_fence(o);  // (as k_vector)
  }
}

#define FA_VEC_DISPATCH(KERNEL, ...)                                                              \
  do {                                                                                            \
    const int g_ = grid_for(mesh->nnodes);                                                        \
    const bool dam_ = F.kind == FA_ASYM_DAMAGE; /* FA_ASYM_DAMAGE_AD maps here, F.ad set */       \
    switch (mesh->cell_type) {                                                                    \
      case FA_TRIANGLE:                                                                           \
        if (dam_) KERNEL<2, 3, FA_ASYM_DAMAGE><<<g_, 256, 0, s>>>(__VA_ARGS__);                   \
        else KERNEL<2, 3, 0><<<g_, 256, 0, s>>>(__VA_ARGS__);                                     \
        break;                                                                                    \
      case FA_QUADRILATERAL: KERNEL<2, 4, 0><<<g_, 256, 0, s>>>(__VA_ARGS__); break;               \
      case FA_TETRAHEDRON: KERNEL<3, 4, 0><<<g_, 256, 0, s>>>(__VA_ARGS__); break;                 \
      case FA_HEXAHEDRON: KERNEL<3, 8, 0><<<g_, 256, 0, s>>>(__VA_ARGS__); break;                  \
    }                                                                                             \
    LAUNCH_CHECK();                                                                               \
  } while (0)

extern "C" int fa_assemble_vector(const fa_mesh* mesh, const fa_form* form, const fa_adjacency* adj, double* b,
                                  void* stream) {
  int rc = check_mesh(mesh);
  if (rc) return rc;
  if (!adj || !adj->ptr || !adj->idx || !b) return fail(FA_E_ARG, "null argument");
  FormView F;
  if ((rc = form_view(mesh, form, F))) return rc;
  DevTables Ts, Tf;
  if ((rc = get_tables(mesh->cell_type, mesh->degree, form->qdeg, &Ts))) return rc;
  if ((rc = get_tables(mesh->cell_type, mesh->degree, 2 * mesh->degree, &Tf))) return rc;
  hipStream_t s = (hipStream_t)stream;
  MeshView M{mesh->cells, mesh->geom, mesh->x, mesh->ncells, mesh->nnodes, mesh->nn, mesh->nv, mesh->gdim};
  if (mesh->nnodes > 0) FA_VEC_DISPATCH(k_vector, M, F, Ts, Tf, adj->ptr, adj->idx, b);
  return FA_OK;
}

extern "C" int fa_apply_lifting(const fa_mesh* mesh, const fa_form* form, const fa_adjacency* adj, double* b,
                                const int8_t* bc, const double* g, const double* x0, double alpha, void* stream) {
  int rc = check_mesh(mesh);
  if (rc) return rc;
  if (!adj || !adj->ptr || !adj->idx || !b || !bc || !g) return fail(FA_E_ARG, "null argument");
  FormView F;
  if ((rc = form_view(mesh, form, F))) return rc;
  DevTables T;
  if ((rc = get_tables(mesh->cell_type, mesh->degree, form->qdeg, &T))) return rc;
  hipStream_t s = (hipStream_t)stream;
  MeshView M{mesh->cells, mesh->geom, mesh->x, mesh->ncells, mesh->nnodes, mesh->nn, mesh->nv, mesh->gdim};
  if (mesh->nnodes > 0) FA_VEC_DISPATCH(k_lifting, M, F, T, adj->ptr, adj->idx, bc, g, x0, alpha, b);
  return FA_OK;
}

__global__ void k_set_bc(double* __restrict__ b, int64_t n, const int8_t* __restrict__ bc, const double* __restrict__ g,
                         const double* __restrict__ x0, double alpha) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    if (bc[i]) b[i] = alpha * (g[i] - (x0 ? x0[i] : 0.0));
}

extern "C" int fa_set_bc(double* b, int64_t ndofs, const int8_t* bc, const double* g, const double* x0, double alpha,
                         void* stream) {
  if (!b || !bc || !g) return fail(FA_E_ARG, "null argument");
  if (ndofs <= 0) return FA_OK;
  k_set_bc<<<grid_for(ndofs), 256, 0, (hipStream_t)stream>>>(b, ndofs, bc, g, x0, alpha);
  LAUNCH_CHECK();
  return FA_OK;
}

// ------------------------------------------------------------------------------------ BSR SpMV
// y = A x over the row window (the Newton driver's Krylov solver): one thread
// per block row, blocks streamed in order.
template <int BS>
__global__ __launch_bounds__(256) void k_bsr_mult(BsrView A, const double* __restrict__ x, double* __restrict__ y) {
  const int64_t base = A.indptr[A.row_begin];
  for (int64_t r = A.row_begin + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < A.row_end;
       r += (int64_t)gridDim.x * blockDim.x) {
    double acc[BS];
#pragma unroll
    for (int i = 0; i < BS; ++i) acc[i] = 0.0;
    for (int64_t k = A.indptr[r]; k < A.indptr[r + 1]; ++k) {
      const double* blk = A.data + (k - base) * BS * BS;
      const int64_t cidx = A.indices[k];
      double xv[BS];
#pragma unroll
      for (int j = 0; j < BS; ++j) xv[j] = x[cidx * BS + j];
#pragma unroll
      for (int i = 0; i < BS; ++i)
#pragma unroll
        for (int j = 0; j < BS; ++j) acc[i] += blk[i * BS + j] * xv[j];
    }
#pragma unroll
    for (int i = 0; i < BS; ++i) y[r * BS + i] = acc[i];
    if constexpr (BS == 2) store_guard2(acc[0], acc[1]);
    else store_guard3(acc[0], acc[1], acc[2]);
  }
}

extern "C" int fa_bsr_mult(const fa_bsr* A, const double* x, double* y, void* stream) {
  if (!A || !A->indptr || !A->indices || !A->data || !x || !y) return fail(FA_E_ARG, "null argument");
  int64_t wb = A->row_begin, we = A->row_end;
  if (we <= wb) { wb = 0; we = A->nrows; }
  BsrView Av{A->indptr, A->indices, A->data, wb, we};
  hipStream_t s = (hipStream_t)stream;
  const int g = grid_for(we - wb);
  if (we <= wb) return FA_OK;
  if (A->bs == 2) k_bsr_mult<2><<<g, 256, 0, s>>>(Av, x, y);
  else if (A->bs == 3) k_bsr_mult<3><<<g, 256, 0, s>>>(Av, x, y);
  else if (A->bs == 1) k_bsr_mult<1><<<g, 256, 0, s>>>(Av, x, y);
  else return fail(FA_E_UNSUPPORTED, "block size %d", A->bs);
  LAUNCH_CHECK();
  return FA_OK;
}

// Diagonal blocks of the row window (block-Jacobi preconditioner of the Newton driver's CG).
__global__ __launch_bounds__(256) void k_bsr_block_diag(BsrView A, int bs, double* __restrict__ out) {
  const int64_t base = A.indptr[A.row_begin];
  for (int64_t r = A.row_begin + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < A.row_end;
       r += (int64_t)gridDim.x * blockDim.x) {
    double* o = out + (r - A.row_begin) * bs * bs;
    for (int i = 0; i < bs * bs; ++i) o[i] = 0.0;
    int64_t lo = A.indptr[r], hi = A.indptr[r + 1];
    while (lo < hi) {  // columns are sorted
      const int64_t mid = (lo + hi) >> 1;
      if (A.indices[mid] < r) lo = mid + 1; else hi = mid;
    }
    if (lo < A.indptr[r + 1] && A.indices[lo] == r)
      for (int i = 0; i < bs * bs; ++i) o[i] = A.data[(lo - base) * bs * bs + i];
  }
}

extern "C" int fa_bsr_block_diag(const fa_bsr* A, double* out, void* stream) {
  if (!A || !A->indptr || !A->indices || !A->data || !out) return fail(FA_E_ARG, "null argument");
  int64_t wb = A->row_begin, we = A->row_end;
  if (we <= wb) { wb = 0; we = A->nrows; }
  if (we <= wb) return FA_OK;
  BsrView Av{A->indptr, A->indices, A->data, wb, we};
  k_bsr_block_diag<<<grid_for(we - wb), 256, 0, (hipStream_t)stream>>>(Av, A->bs, out);
  LAUNCH_CHECK();
  return FA_OK;
}

// ------------------------------------------------------------------------------------ HBM probe
// Measured HBM peak beside the 8 TB/s spec: a grid-stride stream over n doubles with
// 16 B per lane and four independent accesses in flight per lane. mode 0: copy src -> dst (read +
// write), 1: write only (dst = v), 2: read only (src summed into one double per workgroup, dst[block]).
template <int MODE, int ST = 0>
__global__ __launch_bounds__(256) void k_hbm_probe(double* __restrict__ dst, const double* __restrict__ src, int64_t n2,
                                                   double v) {
  typedef double dv2 __attribute__((ext_vector_type(2)));
  dv2* d2 = reinterpret_cast<dv2*>(dst);
  const dv2* s2 = reinterpret_cast<const dv2*>(src);
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  double sum = 0.0;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < n2; t += 4 * stride) {
    dv2 x[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t i = t + u * stride;
      if (MODE != 1 && i < n2) x[u] = __builtin_nontemporal_load(s2 + i);
      else x[u] = dv2{v, v};
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t i = t + u * stride;
      if (i < n2) {
        if (MODE == 2) sum += x[u].x + x[u].y;
        else if (ST == 0) __builtin_nontemporal_store(x[u], d2 + i);
        else d2[i] = x[u];
      }
    }
  }
  if (MODE == 2) {
    __shared__ double red[256];
    red[threadIdx.x] = sum;
    __syncthreads();
    for (int h = 128; h > 0; h >>= 1) {
      if ((int)threadIdx.x < h) red[threadIdx.x] += red[threadIdx.x + h];
      __syncthreads();
    }
    if (threadIdx.x == 0) dst[blockIdx.x] = red[0];
  }
}

// write-pattern variants (measurement): each wave writes SPAN consecutive KiB per round (16 B per
// lane per instruction), rounds grid-strided; LANE64: each lane writes 64 contiguous bytes instead
template <int SPAN, bool NT, bool LANE64>
__global__ __launch_bounds__(256) void k_hbm_write_span(double* __restrict__ dst, int64_t n2, double v) {
  typedef double dv2 __attribute__((ext_vector_type(2)));
  dv2* d2 = reinterpret_cast<dv2*>(dst);
  const int lane = threadIdx.x & 63;
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  const int64_t per = 64 * SPAN;  // dv2 per wave round
  const dv2 x = dv2{v, v};
  for (int64_t base = wave * per; base < n2; base += nwaves * per) {
#pragma unroll
    for (int u = 0; u < SPAN; ++u) {
      const int64_t i = LANE64 ? base + (int64_t)lane * SPAN + u : base + u * 64 + lane;
      if (i < n2) {
        if (NT) __builtin_nontemporal_store(x, d2 + i);
        else d2[i] = x;
      }
    }
  }
}

// one-shot grids (one workgroup per contiguous piece, no grid-stride loop): each workgroup writes
// PER consecutive KiB with 16 B per lane per instruction (LANE32: each lane 32 contiguous bytes)
template <int PER, bool NT, bool LANE32>
__global__ __launch_bounds__(256) void k_hbm_write_oneshot(double* __restrict__ dst, int64_t n2, double v) {
  typedef double dv2 __attribute__((ext_vector_type(2)));
  dv2* d2 = reinterpret_cast<dv2*>(dst);
  const dv2 x = dv2{v, v};
  const int64_t base = (int64_t)blockIdx.x * (PER * 64);  // dv2 per workgroup
#pragma unroll
  for (int u = 0; u < PER / 4; ++u) {
    const int64_t i = LANE32 ? base + 2 * (int64_t)(u * 256 + threadIdx.x) / 2 * 1 + 0 : base + u * 256 + threadIdx.x;
    if (LANE32) {
      const int64_t j = base + (int64_t)(u * 256 + threadIdx.x) * 2;  // covers 2 * 256 dv2 per u: PER / 8 rounds
      if (u < PER / 8) {
        if (j + 1 < n2) {
          if (NT) { __builtin_nontemporal_store(x, d2 + j); __builtin_nontemporal_store(x, d2 + j + 1); }
          else { d2[j] = x; d2[j + 1] = x; }
        }
      }
    } else if (i < n2) {
      if (NT) __builtin_nontemporal_store(x, d2 + i);
      else d2[i] = x;
    }
  }
}

extern "C" int fa_hbm_probe(int32_t mode, double* dst, const double* src, int64_t n, void* stream) {
  if (n <= 0 || (n & 1)) return fail(FA_E_ARG, "n must be positive and even");
  if (!dst || (mode != 1 && !src)) return fail(FA_E_ARG, "null argument");
  if (((uintptr_t)dst | (uintptr_t)src) & 15) return fail(FA_E_ARG, "buffers must be 16-byte aligned");
  hipStream_t s = (hipStream_t)stream;
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const int grid = cus * 8;  // mode 2 writes one double per workgroup: dst holds >= grid doubles
  if (mode == 2 && n < grid) return fail(FA_E_ARG, "read probe needs n >= %d", grid);
  switch (mode) {
    case 0: k_hbm_probe<0><<<grid, 256, 0, s>>>(dst, src, n / 2, 0.0); break;
    case 1: k_hbm_probe<1><<<grid, 256, 0, s>>>(dst, src, n / 2, 1.0); break;
    case 2: k_hbm_probe<2><<<grid, 256, 0, s>>>(dst, src, n / 2, 0.0); break;
    // store-flavour variants of the write / copy streams (measurement): plain stores, larger grids
    case 3: k_hbm_probe<1, 1><<<grid, 256, 0, s>>>(dst, src, n / 2, 1.0); break;
    case 5: k_hbm_probe<0, 1><<<grid, 256, 0, s>>>(dst, src, n / 2, 0.0); break;
    case 6: k_hbm_probe<1, 0><<<grid * 4, 256, 0, s>>>(dst, src, n / 2, 1.0); break;
    case 7: k_hbm_probe<1, 1><<<grid * 4, 256, 0, s>>>(dst, src, n / 2, 1.0); break;
    case 10: k_hbm_write_span<4, true, false><<<grid, 256, 0, s>>>(dst, n / 2, 1.0); break;
    case 11: k_hbm_write_span<4, false, false><<<grid, 256, 0, s>>>(dst, n / 2, 1.0); break;
    case 12: k_hbm_write_span<16, true, false><<<grid, 256, 0, s>>>(dst, n / 2, 1.0); break;
    case 13: k_hbm_write_span<16, false, false><<<grid, 256, 0, s>>>(dst, n / 2, 1.0); break;
    case 14: k_hbm_write_span<4, true, true><<<grid, 256, 0, s>>>(dst, n / 2, 1.0); break;
    case 15: k_hbm_write_span<4, false, true><<<grid, 256, 0, s>>>(dst, n / 2, 1.0); break;
    case 16: k_hbm_write_span<1, true, false><<<grid, 256, 0, s>>>(dst, n / 2, 1.0); break;
    case 17: k_hbm_write_span<1, false, false><<<grid, 256, 0, s>>>(dst, n / 2, 1.0); break;
    case 18: k_hbm_write_span<4, false, false><<<grid / 2, 256, 0, s>>>(dst, n / 2, 1.0); break;
    case 19: k_hbm_write_span<4, false, false><<<grid * 2, 256, 0, s>>>(dst, n / 2, 1.0); break;
    case 20: k_hbm_write_oneshot<4, false, false><<<(unsigned)((n / 2 + 255) / 256), 256, 0, s>>>(dst, n / 2, 1.0); break;
    case 21: k_hbm_write_oneshot<16, false, false><<<(unsigned)((n / 2 + 1023) / 1024), 256, 0, s>>>(dst, n / 2, 1.0); break;
    case 22: k_hbm_write_oneshot<16, true, false><<<(unsigned)((n / 2 + 1023) / 1024), 256, 0, s>>>(dst, n / 2, 1.0); break;
    case 23: k_hbm_write_oneshot<8, false, true><<<(unsigned)((n / 2 + 511) / 512), 256, 0, s>>>(dst, n / 2, 1.0); break;
    case 24: k_hbm_write_oneshot<32, false, false><<<(unsigned)((n / 2 + 2047) / 2048), 256, 0, s>>>(dst, n / 2, 1.0); break;
    default: return fail(FA_E_ARG, "mode %d", mode);
  }
  LAUNCH_CHECK();
  return FA_OK;
}

// Re-check a plan's affine flag against the mesh's current coordinates (a caller that moved the
// vertices after planning): clears FA_PLAN_AFFINE when a tensor cell is no longer a parallelogram /
// parallelepiped, sets it when every cell is. Synchronises `stream`.
extern "C" int fa_plan_check_affine(const fa_mesh* mesh, fa_plan* plan, void* stream) {
  int rc = check_mesh(mesh);
  if (rc) return rc;
  if (!plan) return fail(FA_E_ARG, "null plan");
  if (!(mesh->cell_type == FA_HEXAHEDRON || mesh->cell_type == FA_QUADRILATERAL) || mesh->ncells == 0) return FA_OK;
  hipStream_t s = (hipStream_t)stream;
  MeshView M{mesh->cells, mesh->geom, mesh->x, mesh->ncells, mesh->nnodes, mesh->nn, mesh->nv, mesh->gdim};
  int* dna = nullptr;
  int na_h = 1;
  HIP_TRY(hipMallocAsync((void**)&dna, sizeof(int), s));
  HIP_TRY(hipMemsetAsync(dna, 0, sizeof(int), s));
  if (mesh->gdim == 3) k_check_affine<3><<<grid_for(mesh->ncells), 256, 0, s>>>(M, dna);
  else k_check_affine<2><<<grid_for(mesh->ncells), 256, 0, s>>>(M, dna);
  LAUNCH_CHECK();
  HIP_TRY(hipMemcpyAsync(&na_h, dna, sizeof(int), hipMemcpyDeviceToHost, s));
  HIP_TRY(hipFreeAsync(dna, s));
  HIP_TRY(hipStreamSynchronize(s));
  if (na_h) plan->cell_flags &= ~FA_PLAN_AFFINE;
  else plan->cell_flags |= FA_PLAN_AFFINE;
  return FA_OK;
}

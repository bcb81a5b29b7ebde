/*
 * femasm — MI355X (gfx950) element-stiffness assembly, C ABI.
 *
 * The drop-in boundary for the reference's hot path (SalzmanA/fem-libraries, mechanic2d):
 * the per-cell B^T.D.B quadrature contraction and its scatter into a global sparse matrix.
 * All pointers are DEVICE pointers (hipMalloc / torch.cuda tensors) unless stated; every
 * call is asynchronous on `stream` (a hipStream_t; NULL = the default stream) unless it
 * returns a size the host needs, which is stated per function.  Buffers are owned by the
 * caller; the library allocates only stream-ordered scratch that it frees before returning.
 * Errors: every function returns FA_OK (0) or a negative FA_E_* code and sets a
 * thread-local message readable with fa_last_error().  Calls are re-entrant across streams.
 *
 * Reference interfaces replaced (paths relative to the reference repo):
 *   fa_tabulate_cells    ufcx `tabulate_tensor_float64` of the ffcx-compiled J form
 *                        (form built at FEniCSx/mechanic2d/asym_elasto_damage_model.cc:684-685
 *                        from FEniCSx/mechanic2d/asym_ufl.py:83) and MFEM
 *                        damIntegrator::AssembleElementGrad
 *                        (MFEM/mechanic2d/asym_elasto_damage_model.cc:639-916), batched over cells.
 *   fa_assemble_matrix   dolfinx::fem::assemble_matrix(set_block_fn(A, ADD_VALUES), J_form, {bcl,bcr})
 *                        + fem::set_diagonal(..., 1.0) as called from the setJ callback
 *                        (FEniCSx/mechanic2d/asym_elasto_damage_model.cc:847-862); MFEM
 *                        NonlinearForm::GetGradient driven from :1546.
 *   fa_build_adjacency,  dolfinx::fem::petsc::create_matrix(J_form) — the sparsity pattern of
 *   fa_sparsity_count,   (FEniCSx/mechanic2d/asym_elasto_damage_model.cc:688).
 *   fa_sparsity_fill
 *   fa_assemble_vector   dolfinx::fem::assemble_vector(b, F_form)
 *                        (FEniCSx/mechanic2d/asym_elasto_damage_model.cc:825) and MFEM
 *                        damIntegrator::AssembleElementVector (:559-637).
 *   fa_apply_lifting,    dolfinx::fem::apply_lifting / set_bc as called from setF
 *   fa_set_bc            (FEniCSx/mechanic2d/asym_elasto_damage_model.cc:827, :836).
 */
#ifndef FEMASM_H
#define FEMASM_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FA_OK 0
#define FA_E_ARG (-1)       /* invalid argument (null pointer, bad size) */
#define FA_E_UNSUPPORTED (-2) /* element / form / quadrature combination not implemented */
#define FA_E_HIP (-3)       /* HIP runtime error (launch, allocation) */
#define FA_E_PATTERN (-4)   /* sparsity pattern missing an entry the mesh needs */
#define FA_E_CAPACITY (-5)  /* a row exceeds a kernel capacity (reported with sizes) */

/* dolfinx::mesh::CellType values */
#define FA_TRIANGLE 3
#define FA_QUADRILATERAL 4
#define FA_TETRAHEDRON (-4)
#define FA_HEXAHEDRON 8

/* Form kinds */
#define FA_LINEAR_ELASTICITY 0 /* sigma = lambda tr(eps) I + 2 mu eps  (reference J with d = 0) */
#define FA_ASYM_DAMAGE 1       /* reference mechanic2d damage law, P1 triangles (2-D plane strain) */
#define FA_NEO_HOOKEAN 2       /* compressible neo-Hookean, AD tangent */
#define FA_ASYM_DAMAGE_AD 3    /* FA_ASYM_DAMAGE with the tangent and stress of the reference's USE_AD build:
                                  forward-over-forward AD of its damage potential
                                  (MFEM/mechanic2d/asym_elasto_damage_model.cc:100-204, :752-763) */

/* fa_assemble_matrix flags */
#define FA_GATHER 0x0        /* row-gather: each BSR row computed once, plain coalesced stores */
#define FA_SCATTER 0x1       /* element-scatter with FP64 atomics (dolfinx/PETSc ADD_VALUES shape) */
#define FA_ZERO_FIRST 0x2    /* FA_SCATTER only: zero A->data first (MatZeroEntries) */
#define FA_DETERMINISTIC 0x4 /* FA_GATHER: bit-reproducible values, run to run (see below) */
#define FA_CHECK_ERRORS 0x8  /* validate the pattern and adjacency first (fa_check_pattern, when adj is given),
                                then synchronise `stream` and return FA_E_PATTERN if a kernel found a (row,
                                column) pair or a Dirichlet diagonal missing from the pattern (debugging) */
/* Deterministic assembly (FA_DETERMINISTIC, or FA_PLAN_DETERMINISTIC in plan->cell_flags, which
 * fa_gather_rows honours too): the row gather adds every element contribution v to a block as the
 * 64-bit integer round(v * 2^s_b) (s_b per BLOCK from a bound on the contributions of the cells adding
 * into it, |v 2^s_b| < 2^50) with integer LDS atomics, so each block's sum is exact and the same in any
 * order, then converts it back with one rounding: the values are identical run to run. Every cell
 * adding into block (a, b) holds node a, so a row's values are within ~2^-50 per summand of its own
 * cells' scale, at any stiffness contrast between rows (the per-row 1e-12 bar is tested at contrasts
 * 1e2 .. 1e8, tests/test_gpu_deterministic.py; rounds 4-5 had one scale per row chunk). For linear
 * elasticity with one Poisson ratio on affine simplices and (round 6) affine Q1 / Q2 quadrilaterals and Q1
 * hexahedra (the
 * k_gather_lin kernels) with a positional plan; other forms return FA_E_UNSUPPORTED. (The reference's MFEM integrator is likewise order-fixed: it runs
 * one thread, MFEM/mechanic2d/asym_elasto_damage_model.cc:27.) */

typedef struct {
  int32_t cell_type;     /* FA_TRIANGLE ... */
  int32_t degree;        /* Lagrange degree of the vector space (1, 2, 3) */
  int32_t gdim;          /* geometric dim = topological dim = block size bs (2 or 3) */
  int32_t nn;            /* nodes per cell of the space: dofmap width */
  int64_t ncells;
  int64_t nnodes;        /* number of space nodes (BSR block rows) */
  const int32_t* cells;  /* [ncells][nn] node dofmap, basix local ordering */
  int32_t nv;            /* geometry nodes per cell (P1 / Q1 vertices) */
  int32_t _pad;
  const int32_t* geom;   /* [ncells][nv] geometry dofmap */
  const double* x;       /* [nverts][gdim] vertex coordinates */
} fa_mesh;

typedef struct {
  int32_t kind;          /* FA_LINEAR_ELASTICITY ... */
  int32_t qdeg;          /* quadrature degree; < 0 = the degree UFL estimates for the form */
  const double* E;       /* [ncells] Young's modulus (DG0), or NULL to use lam/mu */
  double nu;             /* Poisson ratio (Constant) when E != NULL */
  const double* lam;     /* [ncells] Lame lambda when E == NULL */
  const double* mu;      /* [ncells] Lame mu when E == NULL */
  const double* u;       /* [nnodes*bs] state (damage, neo-Hookean, residual); may be NULL */
  const double* d;       /* [nnodes] damage (P1) for FA_ASYM_DAMAGE; may be NULL (= 0) */
  const double* f;       /* [nnodes*bs] body force (residual); may be NULL */
} fa_form;

typedef struct {
  int64_t nrows;         /* block rows = mesh nnodes */
  int32_t bs;            /* block size = gdim */
  int32_t _pad;
  int64_t nblocks;       /* indices length */
  const int64_t* indptr; /* [nrows+1] */
  const int32_t* indices;/* [nblocks], sorted per row */
  double* data;          /* blocks of rows [row_begin, row_end): [indptr[row_end]-indptr[row_begin]][bs][bs] */
  int64_t row_begin;     /* row window held by `data` (a row part of the matrix, or the rows a rank */
  int64_t row_end;       /* owns); row_end <= row_begin means the whole matrix [0, nrows) */
} fa_bsr;
/* A row window lets a caller hold the values of a row range only: a rank's owned rows, or a
 * matrix split into several allocations (femasm.la.MatrixCSR parts). */

typedef struct {
  const int64_t* ptr;    /* [nnodes+1] */
  const int32_t* idx;    /* [ncells*nn] flat dofmap positions p = cell*nn + local, sorted per node */
} fa_adjacency;

/* fa_plan.cell_flags */
#define FA_PLAN_AFFINE 0x1   /* every cell of a tensor mesh is a parallelogram / parallelepiped: its
                                hexahedra assemble through the affine row gather (no element-matrix
                                store); otherwise through the MFMA element kernel + block gather */
#define FA_PLAN_DETERMINISTIC 0x2 /* set by the caller: assemblies with this plan (fa_assemble_matrix and
                                     fa_gather_rows) are deterministic, as with FA_DETERMINISTIC */
#define FA_PLAN_ORDER_SEARCH 0x4  /* set by the caller before fa_plan_order: also run the alternating-path
                                     moves of the bank-order search (fewer LDS bank conflicts, config E
                                     ~0.7 % faster per assembly, plan ~8x slower: 1.5 -> 12 s) */
#define FA_PLAN_NEO 0x8           /* set by fa_plan_gather_form for FA_NEO_HOOKEAN: fa_plan_order orders
                                     the slots for the neo-Hookean kernel's item split */

/* Row-chunk plan for the gather kernel (host-computed once per pattern). */
typedef struct {
  int64_t nchunks;
  const int64_t* row_start;  /* device [nchunks+1] */
  int32_t max_blocks;        /* largest block count of a chunk */
  int32_t max_adj;           /* largest adjacency count of a chunk */
  const uint16_t* slots;     /* optional device [ncells*nn][nn]: for adjacency entry j and column
                                node b, the block's position within row j's column list */
  int32_t slot_order;        /* 0: `slots` is that plain map; > 0: fa_plan_order rewrote it for the
                                gather's item order (value = the kernel's column split) */
  int32_t cell_flags;        /* set by fa_plan_gather: FA_PLAN_AFFINE if every cell is affine */
  const int32_t* eadj;       /* positional plan (fa_plan_order with an entry buffer), else NULL:
                                each chunk's adjacency entries in the plan's bank-balanced order;
                                `slots` is then indexed by that position, chunk-relative */
  const int32_t* corder;     /* optional device [nchunks] (fa_plan_locality): the order in which the
                                gather visits its chunks; NULL = row order */
  const void* contrib;       /* optional contribution plan (fa_plan_contrib): P1/P2 simplices with
                                linear elasticity of one Poisson ratio then assemble through the
                                block-owner gather (no per-contribution LDS atomics) */
  const int64_t* chunk_desc; /* optional device [3 * (nchunks + 1)] (fa_plan_chunk_desc, round 6): the
                                store-decoupled gathers' per-chunk arrays in the visiting order, built
                                once per plan instead of at every launch; NULL = built per launch.
                                Rebuild (or set NULL) after changing corder or row_start */
} fa_plan;

const char* fa_last_error(void);
int fa_version(void);

/* Element metadata: nodes per cell and quadrature points for (cell_type, degree, qdeg). */
int fa_element_info(int32_t cell_type, int32_t degree, int32_t qdeg, int32_t* nn, int32_t* nq);

/* Host-only (no device call): whether an element's reference tensor Ahat (default rule for qdeg < 0)
 * is exactly N / D with small integers, i.e. packs into the integer table the store-decoupled gather
 * reads (simplices; affine quadrilaterals and Q1 hexahedra since round 6, e.g. Q2 quads: D = 180);
 * *packed_denom = D, or 0 when it does not pack (that element then assembles through the generic gather)
 * or for Q2 / Q3 hexahedra.
 * *amax = max |Ahat|. Either pointer may be NULL. */
int fa_element_table_info(int32_t cell_type, int32_t degree, int32_t qdeg, int32_t* packed_denom, double* amax);

/* Node -> cell adjacency (transpose of the dofmap): ptr [nnodes+1], idx [ncells*nn]. */
int fa_build_adjacency(const fa_mesh* mesh, int64_t* ptr, int32_t* idx, void* stream);

/* BSR sparsity: pass 1 writes indptr [nnodes+1] and returns the block count in *nblocks
 * (synchronises `stream` to read it); pass 2 fills indices [nblocks] sorted per row. */
int fa_sparsity_count(const fa_mesh* mesh, const fa_adjacency* adj, int64_t* indptr, int64_t* nblocks, void* stream);
int fa_sparsity_fill(const fa_mesh* mesh, const fa_adjacency* adj, const int64_t* indptr, int32_t* indices, void* stream);

/* Validate a sparsity pattern and its adjacency on the device (synchronises `stream`): indptr[0] = 0,
 * indptr monotone, indptr[nnodes] = nblocks; columns in [0, nnodes) and strictly increasing per row;
 * adjacency ptr[nnodes] = ncells*nn, entries of node r sorted, unique and at dofmap positions holding
 * r; every node of every cell present in the rows of the cell's nodes, and no other column (the
 * pattern dolfinx create_matrix builds). FA_E_PATTERN with the failed checks in fa_last_error().
 * The pattern and the adjacency come from rocPRIM sorts and scans (not code this library controls). */
int fa_check_pattern(const fa_mesh* mesh, const fa_adjacency* adj, const int64_t* indptr, const int32_t* indices,
                     int64_t nblocks, void* stream);

/* Gather plan: row chunks whose blocks and adjacency fit the kernel's LDS budget.
 * row_start is a caller-owned device buffer of capacity nnodes+1; nchunks etc. returned
 * in *plan (synchronises `stream`). */
int fa_plan_gather(const fa_mesh* mesh, const fa_adjacency* adj, const fa_bsr* A, int64_t* row_start, fa_plan* plan,
                   void* stream);

/* fa_plan_gather for the kernel of a form kind: FA_NEO_HOOKEAN chunks fill a larger accumulator
 * and aim at 128 adjacency entries (one round of the workgroup's 256 item lanes); other kinds are
 * fa_plan_gather. fa_assemble_matrix refuses a plan whose chunks exceed the form kernel's
 * accumulator (FA_E_ARG). Neo-Hookean forms assemble only with a positional plan (fa_plan_slots +
 * fa_plan_order with an entry buffer). */
int fa_plan_gather_form(const fa_mesh* mesh, int32_t kind, const fa_adjacency* adj, const fa_bsr* A,
                        int64_t* row_start, fa_plan* plan, void* stream);

/* Optional slot map for the gather plan (removes the per-block column search): slots is a
 * caller-owned device buffer of ncells*nn*nn uint16; on success plan->slots points to it.
 * Fails with FA_E_CAPACITY if a row holds more than 65535 blocks. */
int fa_plan_slots(const fa_mesh* mesh, const fa_adjacency* adj, const fa_bsr* A, uint16_t* slots, fa_plan* plan,
                  void* stream);

/* Bank-conflict-aware order for the gather's LDS adds (affine simplices, linear elasticity).
 * Each 16-lane quarter of a wave adds into LDS in passes set by its lanes' slots mod 16
 * (measured, tools/probe/lds_bank_probe.hip). With eadj == NULL, rewrites plan->slots in place so
 * that every lane of a quarter of the kernel's fixed item mapping visits its blocks in an order
 * that spreads each step over the banks; entries hold (b << 10) | position in the row. With eadj
 * (caller-owned device buffer of ncells*nn int32), the plan also chooses which adjacency entries
 * share a quarter (balancing their residues), writes each chunk's entries in that order to eadj,
 * and rewrites plan->slots by position with chunk-relative block positions (plan->eadj = eadj).
 * Sets plan->slot_order; a no-op (slot_order 0) for elements whose gather does not read an
 * ordered map. Run after fa_plan_slots for EVERY plan sharing the slot map (fa_plan_slots
 * rewrites all rows). */
int fa_plan_order(const fa_mesh* mesh, const fa_adjacency* adj, const fa_bsr* A, int32_t* eadj, fa_plan* plan,
                  void* stream);

/* Re-check plan->cell_flags & FA_PLAN_AFFINE against the mesh's CURRENT vertex coordinates (a
 * caller that moved vertices after fa_plan_gather): the affine tensor gather builds each cell's
 * Jacobian from three edge vectors, so a plan must not call a cell affine that no longer is.
 * Synchronises `stream`. A no-op for simplices (always affine). */
int fa_plan_check_affine(const fa_mesh* mesh, fa_plan* plan, void* stream);

/* Chunk visiting order for cache locality: chunks sorted by the Morton key of a point of each
 * chunk (the centroid of the cell of its first adjacency entry), so that chunks the gather runs
 * close in time share cells and their per-cell records stay in L2. corder is a caller-owned device
 * buffer of plan->nchunks int32; on success plan->corder points to it. Any permutation assembles
 * the same matrix (each chunk owns its rows); only the re-reads of the records change. */
int fa_plan_locality(const fa_mesh* mesh, const fa_adjacency* adj, int32_t* corder, fa_plan* plan, void* stream);

/* The chunk arrays the store-decoupled gathers (linear and neo-Hookean) read — per chunk, in the plan's
 * visiting order (plan->corder, or row order): its first block relative to A's row window, its first
 * adjacency entry, and its block and entry counts — into a caller-owned device buffer of
 * 3 * (plan->nchunks + 1) int64, once per plan (plan time, like the slot map); on success
 * plan->chunk_desc points to it and launches skip rebuilding them (config E: 0.21 ms per assembly, a
 * full read of the pattern's row pointer and adjacency pointer arrays). A must be the matrix (row
 * window) the plan was made for. Call it after fa_plan_locality. */
int fa_plan_chunk_desc(const fa_mesh* mesh, const fa_adjacency* adj, const fa_bsr* A, fa_plan* plan, int64_t* buf,
                       void* stream);

/* Block-owner gather (P1/P2 triangles and tetrahedra, linear elasticity with one Poisson ratio).
 * fa_plan_gather_contrib chunks the rows for it (like fa_plan_gather, smaller chunks: at most
 * 256 adjacency entries). fa_plan_contrib_bytes returns the device buffer size the contribution
 * plan of that chunking needs; fa_plan_contrib fills a caller-owned buffer of that size with
 * every chunk's (cell, row node, column node) contributions sorted by destination block and cut
 * into equal lane segments, and sets plan->contrib. The assembly then sums each block's
 * contributions in registers and writes it once (replaces the same dolfinx call as
 * fa_plan_gather: create_matrix + the cell loop of assemble_matrix,
 * FEniCSx/mechanic2d/asym_elasto_damage_model.cc:688, :852-857). */
int fa_plan_gather_contrib(const fa_mesh* mesh, const fa_adjacency* adj, const fa_bsr* A, int64_t* row_start,
                           fa_plan* plan, void* stream);
int fa_plan_contrib_bytes(const fa_mesh* mesh, const fa_adjacency* adj, const fa_bsr* A, const fa_plan* plan,
                          int64_t* bytes, void* stream);
int fa_plan_contrib(const fa_mesh* mesh, const fa_adjacency* adj, const fa_bsr* A, void* buf, int64_t bytes,
                    fa_plan* plan, void* stream);

/* Per-cell element matrices Ae [ncells_out][nn*bs][nn*bs] (dof = node*bs + comp) for cells
 * [c0, c0+ncells_out) — the batched ufcx tabulate_tensor / AssembleElementGrad. */
int fa_tabulate_cells(const fa_mesh* mesh, const fa_form* form, int64_t c0, int64_t ncells_out, double* Ae,
                      void* stream);

/* Global matrix assembly into A (BSR, pattern from fa_sparsity_*). bc: int8 per dof
 * (node*bs+comp) or NULL. Entries in bc rows/columns get no cell contribution and bc
 * diagonal entries are set to `diag` (dolfinx assemble_matrix + set_diagonal).
 * FA_GATHER needs adj and plan; FA_SCATTER needs neither (plan may be NULL). */
int fa_assemble_matrix(const fa_mesh* mesh, const fa_form* form, const fa_adjacency* adj, const fa_plan* plan,
                       const int8_t* bc, double diag, fa_bsr* A, int32_t flags, void* stream);

/* Split gather: fa_assemble_matrix(FA_GATHER) as two calls sharing a caller-owned work buffer
 * of fa_gather_work_bytes() bytes. fa_gather_prepare computes the per-cell records (geometry,
 * material, tangent, constrained-dof masks) for ALL cells; fa_gather_rows then assembles the
 * rows of `plan` (any sub-window of A: several plans over disjoint row ranges may be run in any
 * order, e.g. a rank's interface planes first, their exchange overlapping the interior rows).
 * `bc` must be the same in both calls. Same semantics per row as fa_assemble_matrix; elements /
 * forms without a gather kernel return FA_E_UNSUPPORTED. Neo-Hookean simplex forms prepare the
 * records of the M gather (k_gather_neo), whose plans must be positional (fa_plan_gather_form +
 * fa_plan_slots + fa_plan_order with an entry buffer); another plan is refused with FA_E_ARG
 * (by fa_assemble_matrix too). The library reads no environment variable: results and accepted
 * arguments depend on the arguments only.
 * (Replaces the same dolfinx call, FEniCSx/mechanic2d/asym_elasto_damage_model.cc:852-857, as
 * fa_assemble_matrix.) */
int fa_gather_work_bytes(const fa_mesh* mesh, const fa_form* form, int64_t* bytes);
int fa_gather_prepare(const fa_mesh* mesh, const fa_form* form, const int8_t* bc, void* work, void* stream);
int fa_gather_rows(const fa_mesh* mesh, const fa_form* form, const fa_adjacency* adj, const fa_plan* plan,
                   const int8_t* bc, double diag, const void* work, fa_bsr* A, void* stream);

/* Residual b += int sigma(u):eps(v) dx_q - int f.v dx_{2p} (b is ADDED into, like dolfinx
 * assemble_vector; the reference zeroes it first). sigma term on the form's quadrature degree
 * (the reference's `dxx`), load term on degree 2p (the reference's default `dx`). Node-parallel
 * through the adjacency: deterministic, one write per dof. u / f may be NULL (= 0). */
int fa_assemble_vector(const fa_mesh* mesh, const fa_form* form, const fa_adjacency* adj, double* b, void* stream);

/* dolfinx apply_lifting with one form: b[i] -= alpha * sum_j A_ij (g_j - x0_j) over bc
 * columns j, computed cell by cell with the cell matrices (bc rows i get no contribution;
 * set_bc overwrites them). The reference calls it with alpha = -1
 * (FEniCSx/mechanic2d/asym_elasto_damage_model.cc:827). g, x0 per dof (x0 may be NULL = 0). */
int fa_apply_lifting(const fa_mesh* mesh, const fa_form* form, const fa_adjacency* adj, double* b, const int8_t* bc,
                     const double* g, const double* x0, double alpha, void* stream);

/* b[i] = alpha * (g[i] - x0[i]) on bc dofs (x0 may be NULL). ndofs = nnodes*bs. */
int fa_set_bc(double* b, int64_t ndofs, const int8_t* bc, const double* g, const double* x0, double alpha,
              void* stream);

/* y = A x (block rows of A's window; x, y blocked dof vectors). The Krylov kernel of the Newton
 * driver that consumes the assembled matrix (the reference solves with CG + BoomerAMG,
 * FEniCSx/mechanic2d/asym_elasto_damage_model.cc:717-813). */
int fa_bsr_mult(const fa_bsr* A, const double* x, double* y, void* stream);

/* out[r - row_begin] = the diagonal block of block row r (zeros when absent), [rows, bs, bs]:
 * the block-Jacobi preconditioner of the driver's CG (the reference uses BoomerAMG, :717-813). */
int fa_bsr_block_diag(const fa_bsr* A, double* out, void* stream);

/* Measurement helper (not part of the reference interface): a 16-B-per-lane grid-stride stream
 * over n doubles (n even, 16-B aligned buffers) for the measured HBM peak beside the 8 TB/s spec
 * (SURVEY.md section 8(d)). mode 0: dst = src (copy), 1: dst = 1.0 (write only), 2: read src
 * (dst receives one partial sum per workgroup; n >= 8 * CUs). Asynchronous on `stream`. */
int fa_hbm_probe(int32_t mode, double* dst, const double* src, int64_t n, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* FEMASM_H */

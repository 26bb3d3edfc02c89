// TEST INFRASTRUCTURE ONLY — never linked into the product library.
//
// extern "C" shims over the reference's own CPU code, compiled by oracle/build_ref.sh
// directly from the headers where they lie under /root/reference (nothing is copied
// into this repository).  The output library oracle/_ref/libgala_ref.so is used by
// tests/golden/make_golden.py to generate the golden fixtures and, when present, by
// bench.py's cpu_baseline leg (kind "reference").
//
// Reference code exercised (paths relative to the reference root):
//   readSM_npy32 build path  tests/common.h:331-366 -> CSRCMatrix::build
//                             src/formats/csrc_matrix.h:148-376, set_all 413-421
//   gSpMM + wsumAgg           src/ops/aggregators.h:12-31, 55-127
//   static_ord_col_breakpoints + ord_col_tiling_torch  src/ops/tiling.h:1594-1608, 222-283
//   inplace_sample_graph_ab   src/ops/tiling.h:454-508
//   getMaskSubgraphs + buildTranspose  src/utils/common.h:26-129 (same as tests/common.h:21-124)
//   readSM (Matrix Market)    src/utils/common.h:397-416 -> MtxIO::readMtx src/utils/mtx_io.h:199-499
#include <malloc.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "src/formats/csrc_matrix.h"
#include "src/formats/dense_matrix.h"
#include "src/ops/aggregators.h"
#include "src/ops/tiling.h"
#include "src/utils/common.h"

typedef CSRCMatrix<int, int, float> SM;
typedef DenseMatrix<int, int, float> DM;

template <typename T>
static T *aligned_copy(const T *src, int64_t n) {
    T *p = (T *)aligned_alloc(64, ((n * sizeof(T) + 63) / 64) * 64 + 64);
    if (n) memcpy(p, src, n * sizeof(T));
    return p;
}

extern "C" int ref_csr_build(int nrows, int ncols, int nnz, const int *src, const int *dst,
                             int *rowptr_out, int *col_out, float *val_out) {
    // exactly the readSM_npy32 sequence: aligned row/col id arrays, a value buffer,
    // build(..., CSRC_TYPE::CSR), set_all(1)  (tests/common.h:354-363)
    int *row_ids = aligned_copy(src, nnz);
    int *col_ids = aligned_copy(dst, nnz);
    float *vals = (float *)aligned_alloc(64, ((int64_t)nnz * 4 + 63) / 64 * 64 + 64);
    SM adj;
    adj.build(nrows, ncols, nnz, row_ids, col_ids, vals, CSRC_TYPE::CSR);
    adj.set_all(1);
    memcpy(rowptr_out, adj.offset_ptr(), (int64_t)(nrows + 1) * sizeof(int));
    memcpy(col_out, adj.ids_ptr(), (int64_t)nnz * sizeof(int));
    if (val_out) memcpy(val_out, adj.vals_ptr(), (int64_t)nnz * sizeof(float));
    free(row_ids);
    free(col_ids);
    free(vals);
    return 0;
}

static void import_graph(SM &A, int nrows, int ncols, int nnz, const int *rowptr, const int *col,
                         const float *val) {
    A.import_csr(nrows, ncols, nnz, const_cast<int *>(col), const_cast<float *>(val),
                 const_cast<int *>(rowptr));
}
static void release_graph(SM &A) {  // imported arrays are not owned: detach before ~CSRCMatrix
    A.import_csr(0, 0, 0, nullptr, nullptr, nullptr);
}

extern "C" int ref_gspmm(int nrows, int ncols, int nnz, const int *rowptr, const int *col,
                         const float *val, const float *X, int F, float *Y) {
    // out row r += sum_e val_e * X[col_e]  in CSR order (gSpMM + wsumAgg); Y is the
    // accumulator (caller zero-fills it, as the generated code does)
    SM A;
    import_graph(A, nrows, ncols, nnz, rowptr, col, val);
    DM B, out;
    B.import_mtx(ncols, F, (int64_t)ncols * F, const_cast<float *>(X));
    out.import_mtx(nrows, F, (int64_t)nrows * F, Y);
    gSpMM<DM, SM>(&A, &B, &out, wsumAgg<float, float, int>);
    B.import_mtx(nullptr);
    out.import_mtx(nullptr);
    release_graph(A);
    return 0;
}

extern "C" int ref_col_tile(int nrows, int ncols, int nnz, const int *rowptr, const int *col,
                            const float *val, int cols_per_partition, int max_seg,
                            int *out_rowptr, int *out_col, float *out_val, int *out_bounds) {
    // the emitted COL_TILE transformation (src/codegen/common.h:417-436)
    SM A;
    import_graph(A, nrows, ncols, nnz, rowptr, col, val);
    std::vector<int> bp = static_ord_col_breakpoints<SM>(&A, cols_per_partition);
    const int segments = (int)bp.size() - 1;
    if (segments > max_seg) {
        release_graph(A);
        return -segments;
    }
    auto oi = torch::TensorOptions().dtype(torch::kInt).requires_grad(false);
    auto of = torch::TensorOptions().dtype(torch::kFloat).requires_grad(false);
    torch::Tensor offsets = torch::zeros({(int64_t)(nrows + 1) * segments}, oi);
    torch::Tensor cols = torch::zeros({nnz}, oi);
    torch::Tensor vals = torch::zeros({nnz}, of);
    torch::Tensor bounds = torch::zeros({2 * segments}, oi);
    ord_col_tiling_torch<SM>(bp, offsets, cols, vals, bounds, &A);
    memcpy(out_rowptr, offsets.data_ptr<int>(), (int64_t)(nrows + 1) * segments * sizeof(int));
    memcpy(out_col, cols.data_ptr<int>(), (int64_t)nnz * sizeof(int));
    memcpy(out_val, vals.data_ptr<float>(), (int64_t)nnz * sizeof(float));
    memcpy(out_bounds, bounds.data_ptr<int>(), 2 * segments * sizeof(int));
    release_graph(A);
    return segments;
}

extern "C" int ref_sample_ab(int nrows, int ncols, int nnz, const int *rowptr, const int *col,
                             const float *val, int nsamp, int ra, int rb, int *out_rowptr,
                             int *out_col, float *out_val) {
    SM A;
    // inplace_sample_graph_ab replaces the graph's arrays; hand it private copies
    import_graph(A, nrows, ncols, nnz, aligned_copy(rowptr, nrows + 1), aligned_copy(col, nnz),
                 aligned_copy(val, nnz));
    int *o0 = A.offset_ptr();
    int *c0 = A.ids_ptr();
    float *v0 = A.vals_ptr();
    inplace_sample_graph_ab<SM>(&A, nsamp, ra, rb);
    memcpy(out_rowptr, A.offset_ptr(), (int64_t)(nrows + 1) * sizeof(int));
    memcpy(out_col, A.ids_ptr(), (int64_t)nrows * nsamp * sizeof(int));
    memcpy(out_val, A.vals_ptr(), (int64_t)nrows * nsamp * sizeof(float));
    free(A.offset_ptr());
    free(A.ids_ptr());
    free(A.vals_ptr());
    free(o0);
    free(c0);
    free(v0);
    release_graph(A);
    return 0;
}

extern "C" int ref_mask_subgraphs(int nrows, int nnz, const int *rowptr, const int *col,
                                  const float *mask, int levels, int *out_rowptr, int *out_col,
                                  int *out_nnz, int *t_rowptr, int *t_col) {
    // the emitted SUBGRAPH_DOPT sequence (src/codegen/common.h:480-492): level l of
    // forward_adj / backward_adj; level l's arrays start at l*(nrows+1) and l*nnz
    SM A;
    std::vector<float> ones(nnz, 1.0f);
    import_graph(A, nrows, nrows, nnz, rowptr, col, ones.data());
    DM m;
    m.build(nrows, 1, DM::DENSE_MTX_TYPE::RM, 0);
    memcpy(m.vals_ptr(), mask, (int64_t)nrows * sizeof(float));
    std::vector<SM *> fwd, bwd;
    // getMaskSubgraphs accumulates maxAgg into new_mask->build(nrows, 1, type, 0), which
    // is an uninitialised aligned_alloc (dense_matrix.h:128-141): its result depends on
    // what the heap hands back.  Large graphs get fresh (zero) mmap pages; here glibc's
    // M_PERTURB fills every new allocation with perturb^0xff = 0, so the fixture records
    // the zero-initialised accumulator the code intends.
    mallopt(M_PERTURB, 0xff);
    getMaskSubgraphs<SM, DM>(&A, &m, levels, fwd, bwd);
    mallopt(M_PERTURB, 0);
    for (int l = 0; l < levels; ++l) {
        const int64_t nv = fwd[l]->nvals();
        out_nnz[l] = (int)nv;
        memcpy(out_rowptr + (int64_t)l * (nrows + 1), fwd[l]->offset_ptr(), (int64_t)(nrows + 1) * sizeof(int));
        memcpy(out_col + (int64_t)l * nnz, fwd[l]->ids_ptr(), nv * sizeof(int));
        memcpy(t_rowptr + (int64_t)l * (nrows + 1), bwd[l]->offset_ptr(), (int64_t)(nrows + 1) * sizeof(int));
        memcpy(t_col + (int64_t)l * nnz, bwd[l]->ids_ptr(), nv * sizeof(int));
    }
    release_graph(A);
    return 0;
}

extern "C" int ref_omp_threads(void) { return omp_get_max_threads(); }

// the CPU baseline runs gSpMM on every core the process may use (bench.py picks the count)
extern "C" void ref_set_threads(int n) { omp_set_num_threads(n); }

// Matrix Market: the reference's MtxIO reader (src/utils/mtx_io.h:199-499) -- the COO
// entries in file order, mirrors of (skew-)symmetric files included -- and readSM's CSR
// (src/utils/common.h:397-416: MtxIO -> CSRCMatrix::build(CSR)).  Returns 1 when the file
// has values, 0 for a pattern file, < 0 on a reader error or too small a capacity.
extern "C" int ref_read_mtx(const char *path, int64_t *nrows, int64_t *ncols, int64_t *nvals, int *rows,
                            int *cols, float *vals, int64_t cap) {
    MtxIO<int, int, float> reader;
    if (reader.readMtx(std::string(path)) != IO_INFO::SUCCESS) return -1;
    int nr, nc, nv, size;
    int *r, *c;
    float *v;
    reader.getData(nr, nc, nv, size, r, c, v);
    *nrows = nr;
    *ncols = nc;
    *nvals = nv;
    if (nv > cap) return -2;
    memcpy(rows, r, (int64_t)nv * sizeof(int));
    memcpy(cols, c, (int64_t)nv * sizeof(int));
    if (v && vals) memcpy(vals, v, (int64_t)nv * sizeof(float));
    return v ? 1 : 0;
}

extern "C" int ref_read_sm_mtx(const char *path, int *rowptr, int *col, float *val, int64_t cap_rows,
                               int64_t cap_nnz) {
    SM A;
    readSM<SM>(std::string(path), &A);
    if ((int64_t)A.nrows() + 1 > cap_rows || (int64_t)A.nvals() > cap_nnz) return -2;
    memcpy(rowptr, A.offset_ptr(), ((int64_t)A.nrows() + 1) * sizeof(int));
    memcpy(col, A.ids_ptr(), (int64_t)A.nvals() * sizeof(int));
    if (val && A.vals_ptr()) memcpy(val, A.vals_ptr(), (int64_t)A.nvals() * sizeof(float));
    return A.vals_ptr() ? 1 : 0;
}

// A dense Matrix Market "array" file through the reference's MtxIO (the array branch of
// readMM, src/utils/mtx_io.h:316-363: column-major entries placed row-major), which readDM
// uses when RNPY is not defined (src/utils/common.h:146-183).  Returns 0, < 0 on errors.
extern "C" int ref_read_mtx_dense(const char *path, int64_t *nrows, int64_t *ncols, float *out, int64_t cap) {
    MtxIO<int, int64_t, float> reader;
    if (reader.readMtx(std::string(path)) != IO_INFO::SUCCESS) return -1;
    int nr, nc;
    int64_t nv, size;
    int *r, *c;
    float *v;
    reader.getData(nr, nc, nv, size, r, c, v);
    *nrows = nr;
    *ncols = nc;
    if ((int64_t)nr * nc > cap || !v) return -2;
    memcpy(out, v, (int64_t)nr * nc * sizeof(float));
    return 0;
}

// Host-side graph layout builders of libgala_hip.so (OpenMP, HOST pointers).
//
// These produce exactly the device layout contract the kernels consume and the
// reference builds on the CPU before its H2D copies (codegen/gala.cu:474-593):
//   gala_host_csr_build       <- CSRCMatrix::build      (src/formats/csrc_matrix.h:148-376)
//   gala_host_col_breakpoints <- static_ord_col_breakpoints (src/ops/tiling.h:1594-1608)
//   gala_host_col_tile        <- ord_col_tiling_torch    (src/ops/tiling.h:222-283)
//   gala_host_sample_ab       <- inplace_sample_graph_ab (src/ops/tiling.h:454-508)
//   gala_host_gen_graph       <- generate_rmat           (src/utils/generator.h:36-118)
// Results are deterministic and independent of the thread count (the reference's
// atomic counting sort is not; its per-row column sort makes the CSR identical anyway).
#include <omp.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <string>
#include <vector>

#include "../../include/gala_hip.h"

namespace {

// atomic placement into row buckets, then a per-row sort by (key, input index)
int bucket_sort(int64_t n_buckets, int64_t n, const int32_t *bucket, const int32_t *key,
                int32_t *offsets_out, int32_t *perm_out) {
    std::vector<int64_t> counts(n_buckets + 1, 0);
    for (int64_t i = 0; i < n; ++i) {
        const int32_t b = bucket[i];
        if (b < 0 || b >= n_buckets) return GALA_ERR_GRAPH;
    }
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) __atomic_fetch_add(&counts[bucket[i] + 1], 1, __ATOMIC_RELAXED);
    for (int64_t b = 0; b < n_buckets; ++b) counts[b + 1] += counts[b];
    if (counts[n_buckets] != n) return GALA_ERR_GRAPH;
    std::vector<int64_t> ws(counts.begin(), counts.end() - 1);
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) {
        const int64_t pos = __atomic_fetch_add(&ws[bucket[i]], 1, __ATOMIC_RELAXED);
        perm_out[pos] = (int32_t)i;
    }
#pragma omp parallel for schedule(dynamic, 1024)
    for (int64_t b = 0; b < n_buckets; ++b) {
        int32_t *s = perm_out + counts[b], *e = perm_out + counts[b + 1];
        std::sort(s, e, [key](int32_t x, int32_t y) {
            return key[x] < key[y] || (key[x] == key[y] && x < y);
        });
    }
#pragma omp parallel for schedule(static)
    for (int64_t b = 0; b <= n_buckets; ++b) offsets_out[b] = (int32_t)counts[b];
    return GALA_OK;
}

inline uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ULL;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
    return x ^ (x >> 31);
}
inline uint64_t hash2(uint64_t seed, uint64_t k) { return splitmix64(splitmix64(seed) ^ k); }
inline int64_t bounded(uint64_t h, int64_t n) {
    return (int64_t)(((unsigned __int128)h * (unsigned __int128)n) >> 64);
}
inline double unit(uint64_t h) { return (double)(h >> 11) * (1.0 / 9007199254740992.0); }

}  // namespace

extern "C" int gala_host_csr_build(int64_t n_rows, int64_t n_cols, int64_t nnz,
                                   const int32_t *src, const int32_t *dst, int32_t *rowptr_out,
                                   int32_t *col_out, int32_t *perm_out) {
    if (n_rows < 0 || n_cols < 0 || nnz < 0 || !rowptr_out) return GALA_ERR_INVALID_ARG;
    if (nnz > INT32_MAX || n_rows >= INT32_MAX) return GALA_ERR_UNSUPPORTED;
    if (nnz > 0 && (!src || !dst || !col_out)) return GALA_ERR_INVALID_ARG;
    for (int64_t i = 0; i < nnz; ++i)
        if (dst[i] < 0 || dst[i] >= n_cols) return GALA_ERR_GRAPH;
    std::vector<int32_t> tmp;
    int32_t *perm = perm_out;
    if (!perm) {
        tmp.resize(nnz);
        perm = tmp.data();
    }
    int st = bucket_sort(n_rows, nnz, src, dst, rowptr_out, perm);
    if (st) return st;
#pragma omp parallel for schedule(static)
    for (int64_t k = 0; k < nnz; ++k) col_out[k] = dst[perm[k]];
    return GALA_OK;
}

extern "C" int64_t gala_host_col_breakpoints(int64_t n_cols, int64_t cols_per_partition,
                                             int32_t *out, int64_t max_out) {
    if (n_cols < 0 || cols_per_partition < 1 || !out || max_out < 1) return GALA_ERR_INVALID_ARG;
    int64_t k = 0;
    out[k++] = 0;
    for (int64_t i = 0; i < n_cols; i += cols_per_partition) {
        if (k >= max_out) return GALA_ERR_INVALID_ARG;
        out[k++] = (int32_t)std::min(n_cols, i + cols_per_partition);
    }
    return k;
}

extern "C" int gala_host_col_tile(int64_t n_rows, const int32_t *rowptr, const int32_t *col,
                                  const float *val, int32_t n_seg, const int32_t *breakpoints,
                                  int32_t *out_rowptr, int32_t *out_col, float *out_val,
                                  int32_t *out_bounds) {
    if (n_rows < 0 || n_seg < 1 || !rowptr || !breakpoints || !out_rowptr || !out_bounds)
        return GALA_ERR_INVALID_ARG;
    const int64_t nnz = rowptr[n_rows];
    if (nnz > 0 && (!col || !out_col)) return GALA_ERR_INVALID_ARG;
    if (val && !out_val) return GALA_ERR_INVALID_ARG;
    // per row and segment: [lo, hi) of the (column-sorted) row's edges inside the tile
    int64_t new_nvals = 0;
    std::vector<int32_t> lo(n_rows), hi(n_rows);
    for (int32_t s = 0; s < n_seg; ++s) {
        const int32_t j0 = breakpoints[s], j1 = breakpoints[s + 1];
#pragma omp parallel for schedule(static)
        for (int64_t r = 0; r < n_rows; ++r) {
            const int32_t *b = col + rowptr[r], *e = col + rowptr[r + 1];
            lo[r] = (int32_t)(std::lower_bound(b, e, j0) - col);
            hi[r] = (int32_t)(std::lower_bound(b, e, j1) - col);
        }
        int32_t *orp = out_rowptr + (int64_t)s * (n_rows + 1);
        out_bounds[2 * s] = (int32_t)new_nvals;
        const int64_t seg_start = new_nvals;
        orp[0] = 0;
        for (int64_t r = 0; r < n_rows; ++r) {
            new_nvals += hi[r] - lo[r];
            orp[r + 1] = (int32_t)(new_nvals - seg_start);
        }
#pragma omp parallel for schedule(static)
        for (int64_t r = 0; r < n_rows; ++r) {
            const int64_t o = seg_start + orp[r];
            const int64_t n = hi[r] - lo[r];
            if (n == 0) continue;  // (an empty graph may pass NULL col / val)
            memcpy(out_col + o, col + lo[r], n * sizeof(int32_t));
            if (val) memcpy(out_val + o, val + lo[r], n * sizeof(float));
        }
        out_bounds[2 * s + 1] = (int32_t)new_nvals;
    }
    return GALA_OK;
}

extern "C" int gala_host_sample_ab(int64_t n_rows, const int32_t *rowptr, const int32_t *col,
                                   const float *val, int32_t nsamp, int32_t ra, int32_t rb,
                                   int32_t *out_rowptr, int32_t *out_col, float *out_val) {
    if (n_rows < 0 || nsamp < 0 || !rowptr || !out_rowptr) return GALA_ERR_INVALID_ARG;
    if (n_rows * (int64_t)nsamp > INT32_MAX) return GALA_ERR_UNSUPPORTED;
    if (n_rows * (int64_t)nsamp > 0 && (!col || !out_col)) return GALA_ERR_INVALID_ARG;
    if (val && !out_val) return GALA_ERR_INVALID_ARG;
    for (int64_t r = 0; r < n_rows; ++r)
        if (nsamp > 0 && rowptr[r + 1] == rowptr[r]) return GALA_ERR_GRAPH;
    int bad = 0;
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n_rows; ++i) {
        const int32_t first = rowptr[i];
        const int32_t total = rowptr[i + 1] - first;
        std::vector<int32_t> used(nsamp);
        for (int32_t ji = 0; ji < nsamp; ++ji) used[ji] = first + (ra * ji + rb) % total;
        std::sort(used.begin(), used.end());
        const int64_t o = i * (int64_t)nsamp;
        for (int32_t j = 0; j < nsamp; ++j) {
            if (used[j] < first || used[j] >= first + total) bad = 1;  // negative ra/rb
            out_col[o + j] = col[used[j]];
            if (val) out_val[o + j] = val[used[j]];
        }
        out_rowptr[i + 1] = (int32_t)(o + nsamp);
    }
    out_rowptr[0] = 0;
    return bad ? GALA_ERR_INVALID_ARG : GALA_OK;
}

extern "C" int gala_host_csr_transpose(int64_t n_rows, int64_t n_cols, const int32_t *rowptr,
                                       const int32_t *col, int32_t *out_rowptr, int32_t *out_col,
                                       int32_t *perm) {
    if (n_rows < 0 || n_cols < 0 || !rowptr || !out_rowptr || !perm) return GALA_ERR_INVALID_ARG;
    const int64_t nnz = rowptr[n_rows];
    if (nnz > 0 && (!col || !out_col)) return GALA_ERR_INVALID_ARG;
    std::vector<int32_t> row_of(nnz);
#pragma omp parallel for schedule(static)
    for (int64_t r = 0; r < n_rows; ++r)
        for (int32_t e = rowptr[r]; e < rowptr[r + 1]; ++e) row_of[e] = (int32_t)r;
    // bucket by column, order inside a bucket by source row (then edge id: stable)
    int st = bucket_sort(n_cols, nnz, col, row_of.data(), out_rowptr, perm);
    if (st) return st;
#pragma omp parallel for schedule(static)
    for (int64_t k = 0; k < nnz; ++k) out_col[k] = row_of[perm[k]];
    return GALA_OK;
}

extern "C" int gala_host_gen_graph(int32_t kind, int64_t n, int64_t n_undirected, uint64_t seed,
                                   int32_t *src, int32_t *dst) {
    if (n < 1 || n_undirected < 0 || !src || !dst || kind < 0 || kind > 2) return GALA_ERR_INVALID_ARG;
    if (2 * n_undirected + n > INT32_MAX || n >= INT32_MAX) return GALA_ERR_UNSUPPORTED;
    const double a = 0.57, b = 0.19, c = 0.19;
#pragma omp parallel for schedule(static)
    for (int64_t k = 0; k < n_undirected; ++k) {
        int64_t u, v;
        if (kind == 0) {
            u = bounded(hash2(seed, 2 * (uint64_t)k), n);
            v = n > 1 ? (u + 1 + bounded(hash2(seed, 2 * (uint64_t)k + 1), n - 1)) % n : u;
        } else if (kind == 2) {
            // banded: the other end within band = min(8192, max(16, n / 256)) ids, on the side
            // that stays inside [0, n)
            const int64_t band = std::min<int64_t>(8192, std::max<int64_t>(16, n / 256));
            u = bounded(hash2(seed ^ 0xBA4DULL, 2 * (uint64_t)k), n);
            const int64_t off = 1 + bounded(hash2(seed ^ 0xBA4DULL, 2 * (uint64_t)k + 1), std::min(band, n));
            v = u + off < n ? u + off : (u - off >= 0 ? u - off : u);
        } else {
            // recursive quadrant descent of generate_rmat (generator.h:62-80)
            int64_t sr = 0, er = n - 1, sc = 0, ec = n - 1;
            uint64_t ctr = 0;
            while (sr != er && sc != ec) {
                const double rp = unit(hash2(seed ^ 0x5A5A5A5AULL, ((uint64_t)k << 6) + (ctr++)));
                if (rp < a) {
                    er = (sr + er) / 2;
                    ec = (sc + ec) / 2;
                } else if (rp < a + b) {
                    er = (sr + er) / 2;
                    sc = (sc + ec) / 2;
                } else if (rp < a + b + c) {
                    sr = (sr + er) / 2;
                    ec = (sc + ec) / 2;
                } else {
                    sr = (sr + er) / 2;
                    sc = (sc + ec) / 2;
                }
            }
            u = sr;
            v = sc;
        }
        src[2 * k] = (int32_t)u;
        dst[2 * k] = (int32_t)v;
        src[2 * k + 1] = (int32_t)v;
        dst[2 * k + 1] = (int32_t)u;
    }
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) {
        src[2 * n_undirected + i] = (int32_t)i;
        dst[2 * n_undirected + i] = (int32_t)i;
    }
    return GALA_OK;
}

extern "C" int32_t gala_host_split_threshold(int64_t n_rows, int64_t nnz) {
    if (n_rows < 0 || nnz < 0) return GALA_ERR_INVALID_ARG;
    const int64_t mean_up = (nnz + n_rows - 1) / (n_rows > 0 ? n_rows : 1);  // ceil(nnz / n)
    const int64_t thr = 8 * mean_up > 1024 ? 8 * mean_up : 1024;
    return thr > INT32_MAX ? INT32_MAX : (int32_t)thr;
}

extern "C" int gala_host_split_plan(int64_t n_rows, const int32_t *rowptr, int32_t threshold,
                                    int32_t chunk, int32_t *rows, int32_t *row_chunk0,
                                    int32_t *chunk_row, int64_t *n_rows_split,
                                    int64_t *n_chunks) {
    if (n_rows < 0 || !rowptr || threshold < 1 || chunk < 1 || !n_rows_split || !n_chunks)
        return GALA_ERR_INVALID_ARG;
    const bool fill = rows != nullptr;
    if (fill && (!row_chunk0 || !chunk_row)) return GALA_ERR_INVALID_ARG;
    int64_t cnt = 0, chunks = 0;
    for (int64_t r = 0; r < n_rows; ++r) {
        const int64_t deg = (int64_t)rowptr[r + 1] - rowptr[r];
        if (deg < 0) return GALA_ERR_GRAPH;
        if (deg <= threshold) continue;
        const int64_t nc = (deg + chunk - 1) / chunk;
        if (fill) {
            rows[cnt] = (int32_t)r;
            row_chunk0[cnt] = (int32_t)chunks;
            for (int64_t k = 0; k < nc; ++k) chunk_row[chunks + k] = (int32_t)cnt;
        }
        ++cnt;
        chunks += nc;
    }
    if (chunks > INT32_MAX) return GALA_ERR_UNSUPPORTED;
    if (fill) row_chunk0[cnt] = (int32_t)chunks;
    *n_rows_split = cnt;
    *n_chunks = chunks;
    return GALA_OK;
}

extern "C" int gala_host_row_order(int64_t n_rows, const int32_t *rowptr, int32_t *order) {
    if (n_rows < 0 || (n_rows > 0 && (!rowptr || !order))) return GALA_ERR_INVALID_ARG;
    constexpr int64_t kCap = 4096;
    std::vector<int64_t> start(kCap + 2, 0);
    for (int64_t r = 0; r < n_rows; ++r) {
        const int64_t deg = (int64_t)rowptr[r + 1] - rowptr[r];
        if (deg < 0) return GALA_ERR_GRAPH;
        start[kCap - std::min(deg, kCap) + 1]++;  // bucket 0 = the longest rows
    }
    for (int64_t b = 1; b <= kCap + 1; ++b) start[b] += start[b - 1];
    const int64_t n_capped = start[1];  // rows with deg >= kCap: bucket 0
    for (int64_t r = 0; r < n_rows; ++r) {
        const int64_t deg = (int64_t)rowptr[r + 1] - rowptr[r];
        order[start[kCap - std::min(deg, kCap)]++] = (int32_t)r;
    }
    // bucket 0 in exact descending degree (ties by row id): the whole order is then
    // non-increasing in degree, so its first n entries are exactly the n longest rows -- the
    // hub rows of any threshold (k_spmm_hub_exact takes them from there)
    std::stable_sort(order, order + n_capped, [&](int32_t a, int32_t b) {
        return rowptr[a + 1] - rowptr[a] > rowptr[b + 1] - rowptr[b];
    });
    return GALA_OK;
}

extern "C" int gala_host_mask_subgraph(int64_t n_rows, const int32_t *rowptr, const int32_t *col,
                                       const int32_t *mask, int32_t *out_rowptr,
                                       int32_t *out_col, int32_t *next_mask) {
    // one level of getMaskSubgraphs (tests/common.h:21-110): keep the rows whose mask is
    // set (every edge of such a row, in order), empty the rest; the next level's mask is
    // maxAgg over the full graph, next[i] = max_{e in row i} mask[col_e] (gSpMM + maxAgg,
    // tests/common.h:103-107), with an empty row giving 0 (maxAgg's initial value).
    if (n_rows < 0 || !rowptr || !mask || !out_rowptr) return GALA_ERR_INVALID_ARG;
    const int64_t nnz = rowptr[n_rows];
    if (nnz > 0 && !col) return GALA_ERR_INVALID_ARG;
    out_rowptr[0] = 0;
    for (int64_t r = 0; r < n_rows; ++r) {
        const int64_t d = mask[r] > 0 ? rowptr[r + 1] - rowptr[r] : 0;
        out_rowptr[r + 1] = (int32_t)(out_rowptr[r] + d);
    }
    if (out_col) {
#pragma omp parallel for schedule(dynamic, 1024)
        for (int64_t r = 0; r < n_rows; ++r) {
            if (mask[r] <= 0) continue;
            std::copy(col + rowptr[r], col + rowptr[r + 1], out_col + out_rowptr[r]);
        }
    }
    if (next_mask) {
#pragma omp parallel for schedule(dynamic, 1024)
        for (int64_t r = 0; r < n_rows; ++r) {
            int32_t m = 0;
            for (int32_t e = rowptr[r]; e < rowptr[r + 1]; ++e) m = std::max(m, mask[col[e]]);
            next_mask[r] = m;
        }
    }
    return GALA_OK;
}

// ---- Matrix Market (readSM -> MtxIO::readMM, src/utils/mtx_io.h:199-499) ----------------
namespace {

struct MtxHeader {
    int64_t n_rows = 0, n_cols = 0, nnz = 0;
    int32_t field = 0, symmetry = 0;
    bool dense = false;
};

// Header line "%%MatrixMarket matrix coordinate <field> <symmetry>", then comment lines
// (first character '%'), then the size line "rows cols nnz" -- as readHeaderMM,
// skipCommentsMM and readCooSizeMM parse them (mtx_io.h:199-270).
int mtx_header(std::ifstream &in, MtxHeader &h, bool want_dense = false) {
    std::string line;
    if (std::getline(in, line).eof()) return GALA_ERR_INVALID_ARG;
    char id[64] = {0}, object[64] = {0}, format[64] = {0}, field[64] = {0}, sym[64] = {0};
    if (sscanf(line.c_str(), "%63s %63s %63s %63s %63s", id, object, format, field, sym) != 5)
        return GALA_ERR_INVALID_ARG;
    if (strcmp(object, "matrix") != 0) return GALA_ERR_INVALID_ARG;
    h.dense = strcmp(format, "array") == 0;
    if (!h.dense && strcmp(format, "coordinate") != 0) return GALA_ERR_INVALID_ARG;
    if (h.dense != want_dense) return GALA_ERR_UNSUPPORTED;  // a graph reader on dense data, or back
    if (strcmp(field, "pattern") == 0) h.field = 0;
    else if (strcmp(field, "integer") == 0) h.field = 1;
    else if (strcmp(field, "real") == 0) h.field = 2;
    else if (strcmp(field, "double") == 0) h.field = 3;
    else if (strcmp(field, "complex") == 0) return GALA_ERR_UNSUPPORTED;
    else return GALA_ERR_INVALID_ARG;
    if (strcmp(sym, "general") == 0) h.symmetry = 0;
    else if (strcmp(sym, "symmetric") == 0) h.symmetry = 1;
    else if (strcmp(sym, "skew-symmetric") == 0) h.symmetry = 2;
    else if (strcmp(sym, "hermitian") == 0) return GALA_ERR_UNSUPPORTED;
    else return GALA_ERR_INVALID_ARG;
    if (h.dense && (h.field == 0 || h.symmetry != 0)) return GALA_ERR_UNSUPPORTED;  // mtx_io.h:323-330
    while (!std::getline(in, line).eof())
        if (line.empty() || line[0] != '%') break;
    unsigned long long nr = 0, nc = 0, nz = 0;
    if (h.dense) {  // readArrSizeMM: "rows cols", nvals = rows * cols
        if (sscanf(line.c_str(), "%llu %llu", &nr, &nc) != 2) return GALA_ERR_INVALID_ARG;
        if (nr > (unsigned long long)INT32_MAX || nc > (unsigned long long)INT32_MAX) return GALA_ERR_UNSUPPORTED;
        nz = nr * nc;
    } else if (sscanf(line.c_str(), "%llu %llu %llu", &nr, &nc, &nz) != 3) {
        return GALA_ERR_INVALID_ARG;
    }
    if (nr > (unsigned long long)INT32_MAX || nc > (unsigned long long)INT32_MAX ||
        nz > (unsigned long long)INT64_MAX / 2)
        return GALA_ERR_UNSUPPORTED;
    h.n_rows = (int64_t)nr;
    h.n_cols = (int64_t)nc;
    h.nnz = (int64_t)nz;
    return GALA_OK;
}

}  // namespace

extern "C" int gala_host_mtx_info(const char *path, int64_t *n_rows, int64_t *n_cols, int64_t *nnz,
                                  int32_t *field, int32_t *symmetry, int64_t *capacity) {
    if (!path || !n_rows || !n_cols || !nnz || !field || !symmetry || !capacity) return GALA_ERR_INVALID_ARG;
    std::ifstream in(path);
    if (!in.good()) return GALA_ERR_INVALID_ARG;
    MtxHeader h;
    const int st = mtx_header(in, h);
    if (st != GALA_OK) return st;
    *n_rows = h.n_rows;
    *n_cols = h.n_cols;
    *nnz = h.nnz;
    *field = h.field;
    *symmetry = h.symmetry;
    *capacity = h.symmetry ? 2 * h.nnz : h.nnz;
    return GALA_OK;
}

extern "C" int gala_host_mtx_read(const char *path, int32_t *rows, int32_t *cols, float *vals,
                                  int64_t capacity, int64_t *count_out) {
    if (!path || !rows || !cols || !count_out || capacity < 0) return GALA_ERR_INVALID_ARG;
    std::ifstream in(path);
    if (!in.good()) return GALA_ERR_INVALID_ARG;
    MtxHeader h;
    const int st = mtx_header(in, h);
    if (st != GALA_OK) return st;
    if (capacity < (h.symmetry ? 2 * h.nnz : h.nnz)) return GALA_ERR_INVALID_ARG;
    std::string line;
    int64_t index = 0;
    // readMM's loop (mtx_io.h:404-447): an entry line is used only when getline did not
    // reach the end of the file while reading it
    for (int64_t li = 0; li < h.nnz && !std::getline(in, line).eof(); ++li) {
        long long r = 0, c = 0, iv = 0;
        double dv = 0.0;
        int got;
        if (h.field == 0) got = sscanf(line.c_str(), "%lld %lld", &r, &c) == 2;
        else if (h.field == 1) got = sscanf(line.c_str(), "%lld %lld %lld", &r, &c, &iv) == 3;
        else got = sscanf(line.c_str(), "%lld %lld %lf", &r, &c, &dv) == 3;
        if (!got) return GALA_ERR_INVALID_ARG;
        if (r < 1 || r > h.n_rows || c < 1 || c > h.n_cols) return GALA_ERR_GRAPH;
        const float v = h.field == 0 ? 1.0f : h.field == 1 ? (float)iv : (float)dv;
        rows[index] = (int32_t)(r - 1);
        cols[index] = (int32_t)(c - 1);
        if (vals) vals[index] = v;
        ++index;
        if (h.symmetry && r != c) {  // the mirror, same value (mtx_io.h:435-445)
            if (c > h.n_rows || r > h.n_cols) return GALA_ERR_GRAPH;  // a non-square "symmetric" file
            rows[index] = (int32_t)(c - 1);
            cols[index] = (int32_t)(r - 1);
            if (vals) vals[index] = v;
            ++index;
        }
    }
    *count_out = index;
    return GALA_OK;
}

extern "C" int gala_host_mtx_dense_info(const char *path, int64_t *n_rows, int64_t *n_cols) {
    if (!path || !n_rows || !n_cols) return GALA_ERR_INVALID_ARG;
    std::ifstream in(path);
    if (!in.good()) return GALA_ERR_INVALID_ARG;
    MtxHeader h;
    const int st = mtx_header(in, h, true);
    if (st != GALA_OK) return st;
    *n_rows = h.n_rows;
    *n_cols = h.n_cols;
    return GALA_OK;
}

extern "C" int gala_host_mtx_read_dense(const char *path, float *out, int64_t n_rows, int64_t n_cols,
                                        int64_t *count_out) {
    if (!path || !count_out || n_rows < 0 || n_cols < 0 || (!out && n_rows * n_cols > 0))
        return GALA_ERR_INVALID_ARG;
    std::ifstream in(path);
    if (!in.good()) return GALA_ERR_INVALID_ARG;
    MtxHeader h;
    const int st = mtx_header(in, h, true);
    if (st != GALA_OK) return st;
    if (h.n_rows != n_rows || h.n_cols != n_cols) return GALA_ERR_INVALID_ARG;
    std::fill(out, out + n_rows * n_cols, 0.0f);
    std::string line;
    int64_t index = 0;
    // the array branch of readMM (mtx_io.h:343-363): column-major entries, each line used
    // only when a newline ends it
    for (; index < h.nnz && !std::getline(in, line).eof(); ++index) {
        long long iv = 0;
        double dv = 0.0;
        float v;
        if (h.field == 1) {
            if (sscanf(line.c_str(), "%lld", &iv) != 1) return GALA_ERR_INVALID_ARG;
            v = (float)iv;
        } else {
            if (sscanf(line.c_str(), "%lf", &dv) != 1) return GALA_ERR_INVALID_ARG;
            v = (float)dv;
        }
        out[(index % n_rows) * n_cols + index / n_rows] = v;
    }
    *count_out = index;
    return GALA_OK;
}


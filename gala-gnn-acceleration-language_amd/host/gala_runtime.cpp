// gala_runtime.cpp — host runtime of galac-emitted programs (see gala_runtime.h).
#include "gala_runtime.h"

#include "gala_datasets.h"

#include <hip/hip_runtime_api.h>
#include <unistd.h>
#include <omp.h>
#include <sys/stat.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iostream>
#include <map>
#include <random>
#include <stdexcept>

namespace gala {
namespace rt {

namespace {

void check(int status, const char *fn) {
    TORCH_CHECK(status == GALA_OK, "gala: ", fn, " failed: ", gala_status_string(status));
}

bool file_exists(const std::string &p) {
    struct stat st;
    return ::stat(p.c_str(), &st) == 0;
}

std::string with_slash(std::string d) {
    if (!d.empty() && d.back() != '/') d += '/';
    return d;
}

// ---- .npy reader (format 1.0-3.0, C order, little endian) -----------------------------
struct Npy {
    std::string descr;
    std::vector<int64_t> shape;
    std::vector<char> data;
    int64_t count() const {
        int64_t c = 1;
        for (int64_t s : shape) c *= s;
        return c;
    }
};

std::string header_field(const std::string &h, const std::string &key) {
    const size_t k = h.find("'" + key + "'");
    TORCH_CHECK(k != std::string::npos, "npy header lacks ", key);
    size_t v = h.find(':', k) + 1;
    while (v < h.size() && h[v] == ' ') ++v;
    if (h[v] == '\'') return h.substr(v + 1, h.find('\'', v + 1) - v - 1);
    if (h[v] == '(') return h.substr(v + 1, h.find(')', v) - v - 1);
    size_t e = v;
    while (e < h.size() && h[e] != ',' && h[e] != '}') ++e;
    return h.substr(v, e - v);
}

Npy read_npy(const std::string &path) {
    std::ifstream f(path, std::ios::binary);
    TORCH_CHECK(f, "gala: cannot open ", path);
    char magic[8];
    f.read(magic, 8);
    TORCH_CHECK(f && std::memcmp(magic, "\x93NUMPY", 6) == 0, "gala: ", path, " is not .npy");
    uint32_t hlen = 0;
    if (magic[6] == 1) {
        uint16_t h16;
        f.read((char *)&h16, 2);
        hlen = h16;
    } else {
        f.read((char *)&hlen, 4);
    }
    std::string h(hlen, ' ');
    f.read(&h[0], hlen);
    Npy n;
    n.descr = header_field(h, "descr");
    TORCH_CHECK(header_field(h, "fortran_order").find("False") != std::string::npos,
                "gala: ", path, ": Fortran order not supported");
    const std::string shp = header_field(h, "shape");
    size_t p = 0;
    while (p < shp.size()) {
        while (p < shp.size() && (shp[p] == ' ' || shp[p] == ',')) ++p;
        if (p >= shp.size()) break;
        size_t q = p;
        while (q < shp.size() && std::isdigit((unsigned char)shp[q])) ++q;
        TORCH_CHECK(q > p, "gala: bad npy shape in ", path);
        n.shape.push_back(std::stoll(shp.substr(p, q - p)));
        p = q;
    }
    TORCH_CHECK(n.descr.size() >= 3 && n.descr[0] != '>', "gala: big-endian npy in ", path);
    const int64_t isz = std::stoll(n.descr.substr(2));
    n.data.resize((size_t)(n.count() * isz));
    f.read(n.data.data(), (std::streamsize)n.data.size());
    TORCH_CHECK(f, "gala: truncated npy ", path);
    return n;
}

torch::ScalarType npy_type(const std::string &d) {
    static const std::map<std::string, torch::ScalarType> m = {
        {"f4", torch::kFloat}, {"f8", torch::kDouble}, {"i4", torch::kInt},
        {"i8", torch::kLong},  {"u1", torch::kByte},   {"b1", torch::kBool},
        {"i1", torch::kChar},  {"i2", torch::kShort}};
    const std::string k = d.substr(1);
    if (k == "u4") return torch::kLong;  // widened below
    auto it = m.find(k);
    TORCH_CHECK(it != m.end(), "gala: unsupported npy dtype ", d);
    return it->second;
}

torch::Tensor npy_tensor(const std::string &path) {
    Npy n = read_npy(path);
    std::vector<int64_t> shape(n.shape.begin(), n.shape.end());
    if (n.descr.substr(1) == "u4") {
        auto t = torch::empty(shape, torch::kLong);
        const uint32_t *s = (const uint32_t *)n.data.data();
        int64_t *d = t.data_ptr<int64_t>();
        for (int64_t i = 0; i < n.count(); ++i) d[i] = s[i];
        return t;
    }
    auto t = torch::empty(shape, npy_type(n.descr));
    std::memcpy(t.data_ptr(), n.data.data(), n.data.size());
    return t;
}

// ---- synthetic datasets -----------------------------------------------------------------
DatasetShape shape_of(const std::string &name) {
    DatasetShape s{};
    TORCH_CHECK(dataset_shape(name, &s), "gala: no dataset directory for '", name,
                "' and no synthetic shape known for it (pass --data DIR)");
    return s;
}

inline uint64_t mix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ULL;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
    return x ^ (x >> 31);
}
inline double unit(uint64_t h) { return (double)(h >> 11) * (1.0 / 9007199254740992.0); }

void synthetic_nodes(Dataset &ds, const DatasetShape &s, const RunArgs &a);

Dataset synthetic(const std::string &name, const RunArgs &a, int64_t feat_size,
                  int64_t label_size) {
    DatasetShape s = shape_of(name);
    if (feat_size > 0) s.feat = feat_size;
    if (label_size > 0) s.classes = label_size;
    const int64_t n = std::max<int64_t>(2, (int64_t)std::llround(s.n * a.scale));
    const int64_t und = std::max<int64_t>(1, (int64_t)std::llround(s.undirected * a.scale));
    const int64_t m = 2 * und + n;
    std::vector<int32_t> src(m), dst(m);
    check(gala_host_gen_graph(0, n, und, 42 + a.seed, src.data(), dst.data()),
          "gala_host_gen_graph");
    Dataset ds;
    ds.name = name;
    ds.source = "synthetic";
    ds.n = n;
    ds.rowptr = torch::empty({n + 1}, torch::kInt);
    ds.col = torch::empty({m}, torch::kInt);
    check(gala_host_csr_build(n, n, m, src.data(), dst.data(), ds.rowptr.data_ptr<int32_t>(),
                              ds.col.data_ptr<int32_t>(), nullptr),
          "gala_host_csr_build");
    synthetic_nodes(ds, s, a);
    return ds;
}

// Seeded features U[-1, 1), labels and train / valid / test masks of the dataset's shape for
// the ds.n vertices of ds (a synthetic graph, or a Matrix Market graph without node data).
void synthetic_nodes(Dataset &ds, const DatasetShape &s, const RunArgs &a) {
    const int64_t n = ds.n;
    ds.feat = torch::empty({n, s.feat}, torch::kFloat);
    float *fp = ds.feat.data_ptr<float>();
    const uint64_t fseed = mix64(0xFEA7ULL + a.seed);
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n * s.feat; ++i)
        fp[i] = (float)(2.0 * unit(mix64(fseed ^ (uint64_t)i)) - 1.0);
    ds.labels = torch::empty({n}, torch::kLong);
    ds.train_mask = torch::empty({n}, torch::kBool);
    ds.valid_mask = torch::empty({n}, torch::kBool);
    ds.test_mask = torch::empty({n}, torch::kBool);
    int64_t *lp = ds.labels.data_ptr<int64_t>();
    bool *tr = ds.train_mask.data_ptr<bool>(), *va = ds.valid_mask.data_ptr<bool>(),
         *te = ds.test_mask.data_ptr<bool>();
    const uint64_t lseed = mix64(0x1AB5ULL + a.seed), mseed = mix64(0x3A5CULL + a.seed);
    for (int64_t i = 0; i < n; ++i) {
        lp[i] = (int64_t)(mix64(lseed ^ (uint64_t)i) % (uint64_t)s.classes);
        const double u = unit(mix64(mseed ^ (uint64_t)i));
        tr[i] = u < s.train;
        va[i] = !tr[i] && u < s.train + s.valid;
        te[i] = !tr[i] && !va[i];
    }
    ds.classes = s.classes;
}

// A Matrix Market graph (the reference's readSM -> MtxIO, src/utils/common.h:397-416;
// gala_host_mtx_read), its pattern as the adjacency; node data synthetic of the program's
// dataset shape (feature / label sizes from the program).
Dataset from_mtx(const std::string &name, const std::string &path, const RunArgs &a, int64_t feat_size,
                 int64_t label_size) {
    int64_t nr = 0, nc = 0, nnz = 0, cap = 0;
    int32_t field = 0, sym = 0;
    check(gala_host_mtx_info(path.c_str(), &nr, &nc, &nnz, &field, &sym, &cap), "gala_host_mtx_info");
    TORCH_CHECK(nr == nc, "gala: non-square Matrix Market graph ", path);
    std::vector<int32_t> rows(std::max<int64_t>(cap, 1)), cols(std::max<int64_t>(cap, 1));
    int64_t m = 0;
    check(gala_host_mtx_read(path.c_str(), rows.data(), cols.data(), nullptr, cap, &m), "gala_host_mtx_read");
    Dataset ds;
    ds.name = name;
    ds.source = path;
    ds.n = nr;
    ds.rowptr = torch::empty({nr + 1}, torch::kInt);
    ds.col = torch::empty({m}, torch::kInt);
    check(gala_host_csr_build(nr, nc, m, rows.data(), cols.data(), ds.rowptr.data_ptr<int32_t>(),
                              ds.col.data_ptr<int32_t>(), nullptr),
          "gala_host_csr_build");
    DatasetShape s{};
    if (!dataset_shape(name, &s)) s = DatasetShape{nr, 0, 16, 2, 0.5, 0.2};
    if (feat_size > 0) s.feat = feat_size;
    if (label_size > 0) s.classes = label_size;
    synthetic_nodes(ds, s, a);
    return ds;
}

Dataset from_files(const std::string &name, const std::string &dir, int64_t feat_size,
                   int64_t label_size) {
    Dataset ds;
    ds.name = name;
    ds.source = dir;
    // readSM_npy32 (tests/common.h:331-366): Adj_src = [nrows, ncols, src...]
    auto src = npy_tensor(dir + "Adj_src.npy").to(torch::kLong).view(-1);
    auto dst = npy_tensor(dir + "Adj_dst.npy").to(torch::kLong).view(-1);
    TORCH_CHECK(src.numel() >= 2 && src.numel() - 2 == dst.numel(), "gala: ", dir,
                "Adj_src.npy / Adj_dst.npy sizes disagree");
    const int64_t nrows = src[0].item<int64_t>(), ncols = src[1].item<int64_t>();
    TORCH_CHECK(nrows == ncols, "gala: non-square adjacency in ", dir);
    const int64_t m = dst.numel();
    // ids are range-checked before the int32 narrowing (a wrapped id could otherwise land on
    // a valid-looking vertex and silently build another graph)
    TORCH_CHECK(nrows >= 0 && nrows < INT32_MAX, "gala: ", dir, "Adj_src.npy: ", nrows,
                " vertices exceed the int32 index contract");
    if (m > 0) {
        auto s = src.slice(0, 2);
        TORCH_CHECK(s.min().item<int64_t>() >= 0 && s.max().item<int64_t>() < nrows &&
                        dst.min().item<int64_t>() >= 0 && dst.max().item<int64_t>() < ncols,
                    "gala: ", dir, "Adj_src.npy / Adj_dst.npy hold vertex ids outside [0, ", nrows, ")");
    }
    auto s32 = src.slice(0, 2).to(torch::kInt).contiguous();
    auto d32 = dst.to(torch::kInt).contiguous();
    ds.n = nrows;
    ds.rowptr = torch::empty({nrows + 1}, torch::kInt);
    ds.col = torch::empty({m}, torch::kInt);
    check(gala_host_csr_build(nrows, ncols, m, s32.data_ptr<int32_t>(), d32.data_ptr<int32_t>(),
                              ds.rowptr.data_ptr<int32_t>(), ds.col.data_ptr<int32_t>(), nullptr),
          "gala_host_csr_build");
    ds.feat = npy_tensor(dir + "Feat.npy").to(torch::kFloat).contiguous();
    TORCH_CHECK(ds.feat.dim() == 2 && ds.feat.size(0) == nrows, "gala: Feat.npy shape");
    TORCH_CHECK(feat_size <= 0 || ds.feat.size(1) == feat_size, "gala: Feat.npy has ",
                ds.feat.size(1), " columns but the program says feature_size(", feat_size, ")");
    ds.labels = npy_tensor(dir + "Lab.npy").to(torch::kLong).view(-1).contiguous();
    ds.train_mask = npy_tensor(dir + "TnMsk.npy").view(-1).ne(0);
    ds.valid_mask = npy_tensor(dir + "VlMsk.npy").view(-1).ne(0);
    ds.test_mask = npy_tensor(dir + "TsMsk.npy").view(-1).ne(0);
    // classes = max label + 1 (gala.cu:505-507)
    ds.classes = ds.labels.max().item<int64_t>() + 1;
    if (label_size > ds.classes) ds.classes = label_size;
    return ds;
}

struct HostCsr {
    int64_t n_rows = 0, n_cols = 0;
    std::vector<int32_t> rowptr, col;
    int64_t nnz() const { return rowptr.empty() ? 0 : rowptr.back(); }
};

HostCsr transpose(const HostCsr &g, std::vector<int32_t> *perm_out) {
    HostCsr t;
    t.n_rows = g.n_cols;
    t.n_cols = g.n_rows;
    t.rowptr.resize(g.n_cols + 1);
    t.col.resize(g.nnz());
    std::vector<int32_t> perm(g.nnz());
    check(gala_host_csr_transpose(g.n_rows, g.n_cols, g.rowptr.data(), g.col.data(),
                                  t.rowptr.data(), t.col.data(), perm.data()),
          "gala_host_csr_transpose");
    if (perm_out) *perm_out = std::move(perm);
    return t;
}

// Device copy of one CSR, column-tiled if asked (ord_col_tiling_torch layout).
struct DevGraph {
    torch::Tensor off, cols, vals, bounds;
    int segs = 1;
};

DevGraph upload(const HostCsr &g, int64_t col_tile, torch::Device dev) {
    DevGraph d;
    auto io = torch::TensorOptions().dtype(torch::kInt);
    const int64_t nnz = g.nnz();
    if (col_tile > 0) {
        std::vector<int32_t> bp(g.n_cols / std::max<int64_t>(col_tile, 1) + 3);
        const int64_t nbp = gala_host_col_breakpoints(g.n_cols, col_tile, bp.data(), (int64_t)bp.size());
        TORCH_CHECK(nbp >= 2, "gala: gala_host_col_breakpoints failed");
        const int segs = (int)(nbp - 1);
        if (segs > 1) {
            auto off = torch::empty({(g.n_rows + 1) * segs}, io);
            auto cols = torch::empty({nnz}, io);
            auto vals = torch::empty({nnz}, torch::kFloat);
            auto bounds = torch::empty({2 * segs}, io);
            check(gala_host_col_tile(g.n_rows, g.rowptr.data(), g.col.data(), nullptr, segs,
                                     bp.data(), off.data_ptr<int32_t>(), cols.data_ptr<int32_t>(),
                                     vals.data_ptr<float>(), bounds.data_ptr<int32_t>()),
                  "gala_host_col_tile");
            d.off = off.to(dev);
            d.cols = cols.to(dev);
            d.vals = torch::ones({nnz}, torch::TensorOptions().dtype(torch::kFloat).device(dev));
            d.bounds = bounds;
            d.segs = segs;
            return d;
        }
    }
    // .to(dev, ..., copy=true): on the CPU device a plain .to() would alias the host vectors
    d.off = torch::from_blob((void *)g.rowptr.data(), {g.n_rows + 1}, io).to(dev, torch::kInt, false, true);
    d.cols = torch::from_blob((void *)g.col.data(), {nnz}, io).to(dev, torch::kInt, false, true);
    d.vals = torch::ones({nnz}, torch::TensorOptions().dtype(torch::kFloat).device(dev));
    return d;
}

struct Sampling {
    int64_t nsamples = 0;
    bool dynamic = false;
    std::mt19937_64 rng;
} g_sampling;

}  // namespace

RunArgs parse_args(int argc, char **argv) {
    RunArgs a;
    for (int i = 1; i < argc; ++i) {
        const std::string k = argv[i];
        auto val = [&]() -> std::string {
            TORCH_CHECK(i + 1 < argc, "gala: ", k, " needs a value");
            return argv[++i];
        };
        if (k == "--data") {  // a dataset directory, or a Matrix Market graph file
            a.data_dir = val();
            if (a.data_dir.size() < 4 || a.data_dir.compare(a.data_dir.size() - 4, 4, ".mtx") != 0)
                a.data_dir = with_slash(a.data_dir);
        }
        else if (k == "--synthetic") a.synthetic = true;
        else if (k == "--scale") a.scale = std::stod(val());
        else if (k == "--iters") a.iters = std::stoll(val());
        else if (k == "--seed") a.seed = std::stoull(val());
        else if (k == "--dump") a.dump_path = val();
        else if (k == "--quiet") a.quiet = true;
        else if (k == "--device") a.device = val();
        else TORCH_CHECK(false, "gala: unknown option ", k);
    }
    TORCH_CHECK(a.scale > 0, "gala: --scale must be positive");
    TORCH_CHECK(a.device == "gpu" || a.device == "cpu", "gala: --device must be gpu or cpu");
    return a;
}

torch::Device device(const RunArgs &args) {
    if (args.device == "cpu") return torch::Device(torch::kCPU);
    TORCH_CHECK(torch::cuda::is_available(), "gala: no GPU visible (run with --device cpu for "
                "the host backend; there is no silent fallback)");
    return torch::Device(torch::kCUDA, 0);
}

void sync(const torch::Device &dev) {
    if (dev.is_cuda()) torch::cuda::synchronize();
}

Dataset load_dataset(const std::string &name, const RunArgs &args, int64_t feat_size,
                     int64_t label_size, const std::string &opt_input) {
    if (!args.synthetic) {
        const std::string &d0 = args.data_dir;
        if (d0.size() >= 4 && d0.compare(d0.size() - 4, 4, ".mtx") == 0)
            return from_mtx(name, d0, args, feat_size, label_size);
        std::vector<std::string> dirs;
        if (!args.data_dir.empty()) dirs.push_back(args.data_dir);
        if (!opt_input.empty()) dirs.push_back(with_slash(opt_input));
        dirs.push_back("Data/" + name + "/");
        for (const auto &d : dirs)
            if (file_exists(d + "Adj_src.npy")) return from_files(name, d, feat_size, label_size);
        TORCH_CHECK(args.data_dir.empty(), "gala: ", args.data_dir, "Adj_src.npy not found");
    }
    return synthetic(name, args, feat_size, label_size);
}

int prepare_graphs(const Dataset &ds, const GraphPlan &plan, torch::Device dev) {
    HostCsr base;
    base.n_rows = base.n_cols = ds.n;
    base.rowptr.assign(ds.rowptr.data_ptr<int32_t>(), ds.rowptr.data_ptr<int32_t>() + ds.n + 1);
    base.col.assign(ds.col.data_ptr<int32_t>(), ds.col.data_ptr<int32_t>() + base.rowptr.back());
    if (plan.data_sample > 0) {
        // inplace_sample_graph_ab(&adj0, n, 5, 7) (codegen/common.h:493-497)
        const int32_t ns = (int32_t)plan.data_sample;
        HostCsr s;
        s.n_rows = s.n_cols = ds.n;
        s.rowptr.resize(ds.n + 1);
        s.col.resize((size_t)ds.n * ns);
        std::vector<float> sv(s.col.size());
        check(gala_host_sample_ab(ds.n, base.rowptr.data(), base.col.data(), nullptr, ns, 5, 7,
                                  s.rowptr.data(), s.col.data(), sv.data()),
              "gala_host_sample_ab");
        base = std::move(s);
    }
    std::vector<HostCsr> graphs{base};
    if (plan.subgraph_levels > 0) {
        // getMaskSubgraphs (tests/common.h:21-110): level l = rows within l hops of the
        // train mask; aggregation c of L uses level L-1-c (codegen/common.h:484-491)
        const int L = plan.subgraph_levels;
        std::vector<int32_t> mask(ds.n), next(ds.n);
        const bool *tm = ds.train_mask.data_ptr<bool>();
        for (int64_t i = 0; i < ds.n; ++i) mask[i] = tm[i] ? 1 : 0;
        std::vector<HostCsr> levels;
        for (int l = 0; l < L; ++l) {
            HostCsr s;
            s.n_rows = s.n_cols = ds.n;
            s.rowptr.resize(ds.n + 1);
            check(gala_host_mask_subgraph(ds.n, base.rowptr.data(), base.col.data(), mask.data(),
                                          s.rowptr.data(), nullptr, nullptr),
                  "gala_host_mask_subgraph");
            s.col.resize(s.rowptr.back());
            check(gala_host_mask_subgraph(ds.n, base.rowptr.data(), base.col.data(), mask.data(),
                                          s.rowptr.data(), s.col.data(), next.data()),
                  "gala_host_mask_subgraph");
            levels.push_back(std::move(s));
            mask.swap(next);
        }
        for (int c = 0; c < L; ++c) graphs.push_back(levels[L - 1 - c]);
    }
    auto &S = global_slots();
    S.clear();
    for (size_t g = 0; g < graphs.size(); ++g) {
        // a subgraph is never symmetric: its backward is always the transpose
        // (buildTranspose, tests/common.h:112-124)
        const bool same = plan.undirected && g == 0;
        std::vector<int32_t> perm;
        DevGraph fw = upload(graphs[g], plan.col_tile, dev);
        S.push(fw.off, fw.cols, fw.vals, fw.bounds, fw.segs, plan.weighted);
        if (same && !plan.transpose_perm) {
            S.push(fw.off, fw.cols, fw.vals, fw.bounds, fw.segs, plan.weighted);
        } else {
            HostCsr t = transpose(graphs[g], &perm);
            DevGraph bw = upload(t, plan.col_tile, dev);
            const int idx = S.push(bw.off, bw.cols, bw.vals, bw.bounds, bw.segs, plan.weighted);
            if (plan.transpose_perm) {
                TORCH_CHECK(bw.segs == 1, "gala: FIXED-mode GAT needs an untiled graph");
                S.transpose_perm[idx] =
                    torch::from_blob(perm.data(), {(int64_t)perm.size()}, torch::kInt)
                        .to(dev, torch::kInt, false, true);
            }
        }
    }
    S.nrows = ds.n;
    return (int)graphs.size();
}

void set_kernel_sampling(int64_t nsamples, bool dynamic, uint64_t seed) {
    auto &S = global_slots();
    g_sampling.nsamples = nsamples;
    g_sampling.dynamic = dynamic;
    g_sampling.rng.seed(seed);
    S.nsamples = (int)nsamples;
    S.ra = 5;
    S.rb = 7;
}

void next_forward() {
    if (!g_sampling.dynamic) return;
    // std::uniform_int_distribution<>(0, 100) for global_ra / global_rb
    // (codegen/common.h:822-833); seeded here so runs are reproducible
    std::uniform_int_distribution<int> d(0, 100);
    auto &S = global_slots();
    S.ra = d(g_sampling.rng);
    S.rb = d(g_sampling.rng);
}

torch::Tensor sampled_degrees(int64_t nsamples) {
    auto &S = global_slots();
    TORCH_CHECK(!S.offset_graph.empty(), "gala: no graph registered");
    return torch::full({S.nrows, 1}, (float)(nsamples * S.segments[0]),
                       torch::TensorOptions().dtype(torch::kFloat).device(S.offset_graph[0].device()));
}

torch::Tensor degrees() {
    auto &S = global_slots();
    TORCH_CHECK(!S.offset_graph.empty(), "gala: no graph registered");
    return degree_norm(S.offset_graph[0], S.bounds[0], S.segments[0], 1.0, S.columns_graph[0]);
}

torch::Tensor cross_entropy(const torch::Tensor &pred, const torch::Tensor &labels) {
    return -torch::log_softmax(pred, 1).gather(1, labels.reshape({-1, 1}).to(torch::kLong)).mean();
}

double get_time() { return omp_get_wtime(); }

double calc_mean(const std::vector<double> &v) {
    if (v.empty()) return 0.0;
    double s = 0;
    for (double x : v) s += x;
    return s / (double)v.size();
}

int64_t device_memory_mb(const torch::Device &dev) {
    if (!dev.is_cuda()) {
        std::ifstream f("/proc/self/statm");
        int64_t pages = 0, rss = 0;
        if (!(f >> pages >> rss)) return -1;
        return rss * (int64_t)sysconf(_SC_PAGESIZE) / (1024 * 1024);
    }
    size_t free_b = 0, total_b = 0;
    if (hipMemGetInfo(&free_b, &total_b) != hipSuccess) return -1;
    return (int64_t)((total_b - free_b) / (1024 * 1024));
}

void dump(const std::string &path,
          const std::vector<std::pair<std::string, torch::Tensor>> &tensors) {
    std::ofstream f(path, std::ios::binary);
    TORCH_CHECK(f, "gala: cannot write ", path);
    f.write("GALADMP1", 8);
    const uint32_t n = (uint32_t)tensors.size();
    f.write((const char *)&n, 4);
    for (const auto &kv : tensors) {
        torch::Tensor t = kv.second.detach().to(torch::kCPU).contiguous();
        uint8_t code;
        switch (t.scalar_type()) {
        case torch::kFloat: code = 0; break;
        case torch::kLong: code = 1; break;
        case torch::kInt: code = 2; break;
        case torch::kBool: code = 3; break;
        default: t = t.to(torch::kFloat); code = 0;
        }
        const uint32_t nl = (uint32_t)kv.first.size(), nd = (uint32_t)t.dim();
        f.write((const char *)&nl, 4);
        f.write(kv.first.data(), nl);
        f.write((const char *)&code, 1);
        f.write((const char *)&nd, 4);
        for (int64_t d : t.sizes()) f.write((const char *)&d, 8);
        f.write((const char *)t.data_ptr(), (std::streamsize)t.nbytes());
    }
}

}  // namespace rt
}  // namespace gala

// gala_datasets.h — published shapes of the datasets GALA programs load by name.
//
// (N, undirected edges) after gala_export_npy.py's self-loop normalisation (SURVEY.md §8
// dataset table), feature / class counts as in the reference DSL programs
// (tests/GALA-DSL/<model>/<dataset>/h100.txt feature_size / label_size), train / valid
// fractions as DGL / OGB split them.  Used by galac for programs that give no
// feature_size / label_size, and by the runtime to synthesise a dataset's shape when its
// files are absent.  Plain C++ (no torch).
#pragma once

#include <cstdint>
#include <string>

namespace gala {

struct DatasetShape {
    int64_t n, undirected, feat, classes;
    double train, valid;  // split fractions (the rest is test)
};

// false if the name is unknown; papers100M_<p> is the p% node subgraph
// (get_large_sampled_datasets.py:68; an induced subgraph keeps ~p^2 of the edges)
inline bool dataset_shape(const std::string &name, DatasetShape *out) {
    struct Entry {
        const char *name;
        DatasetShape s;
    };
    static const Entry table[] = {
        {"Cora", {2708, 5278, 1433, 7, 140.0 / 2708, 500.0 / 2708}},
        {"Pubmed", {19717, 44324, 500, 3, 60.0 / 19717, 500.0 / 19717}},
        {"CoraFull", {19793, 63421, 8710, 70, 0.70, 0.15}},
        {"Arxiv", {169343, 583122, 128, 40, 0.537, 0.176}},
        {"Products", {2449029, 61859140, 100, 47, 0.080, 0.016}},
        {"Reddit", {232965, 57307946, 602, 41, 0.660, 0.102}},
    };
    for (const Entry &e : table)
        if (name == e.name) {
            *out = e.s;
            return true;
        }
    const std::string pre = "papers100M_";
    if (name.rfind(pre, 0) == 0 && name.size() > pre.size()) {
        const double p = std::stod(name.substr(pre.size())) / 100.0;
        *out = {(int64_t)(111059956 * p), (int64_t)(807842936 * p * p), 128, 172, 0.011, 0.001};
        return true;
    }
    return false;
}

}  // namespace gala

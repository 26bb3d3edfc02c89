// hip.h -- the HIP code generator for the reference compiler: a CodeGenerator subclass
// (src/codegen/common.h:1725-1764) that takes the place of CUDAGenerator
// (src/codegen/cuda.h:10-1400) in the reference's drivers.  A maintainer drops this file
// next to cuda.h and swaps one line of tests/gala_inference.cpp:174-175:
//
//     auto genCode = HIPGenerator(ctx, outputPath);   // was CUDAGenerator
//
// Nothing else in the reference changes: the front-end, the IR, the middle-end passes and
// the base generator's model / autograd / training-loop code stay as they are.  What the
// subclass replaces is what CUDAGenerator adds on top of the base:
//   initCMake   CMake for a host C++ program over libgala_torch.so (no nvcc, no CUDA
//               toolkit, no cuSPARSE);
//   initKernels instead of CUDA kernel sources and launch wrappers (cuda.h:170-955), the
//               emitted `<kernel name>_call` free functions the base's autograd classes
//               call (common.h:622-1127) forward to the operator mirror (host/gala_torch.h),
//               whose kernels are the gfx950 HIP kernels of libgala_hip.so (or, for host
//               tensors, libgala_cpu.so);
//   dataPrep    the graph slots, features, labels and masks become torch tensors on the
//               program's device (torch-owned memory, no cudaMalloc / from_blob leaks), and
//               each graph is registered with the mirror (hub-row plans);
//   writeCode   the base's sections, with its two device-specific spellings (a tensor
//               option `.device(torch::kCUDA, 0)` and `cudaDeviceSynchronize()`, common.h
//               :686-1557) retargeted to the program's device, and an optional dump of the
//               first epoch's prediction, the initial weights, the loss and the weight
//               gradients (GALA_DUMP=<file>); the hidden Linears' calls go to the
//               mirror's FFN op (row-split weight gradients, see denseOnMatrixCores).
// The device is GALA_DEVICE (default "cuda", the HIP device of PyTorch-ROCm; "cpu" runs
// the same program on the host backend).
#ifndef GALA_HIP_CODEGEN_H
#define GALA_HIP_CODEGEN_H

#include <cstdlib>
#include <regex>
#include <unordered_set>

#include "common.h"

class HIPGenerator : public CodeGenerator {
public:
    HIPGenerator(GALAContext *context, std::string &outputPath) : CodeGenerator(context, outputPath) {}

    void initCMake() override {
        std::string cm =
            "cmake_minimum_required(VERSION 3.18)\n"
            "project(gala_hip LANGUAGES CXX)\n"
            "# the generated program is host C++: its kernels are libgala_hip.so's, reached through\n"
            "# the operator mirror libgala_torch.so (GALA_AMD_ROOT: the MI355X backend's checkout)\n"
            "find_package(Torch REQUIRED)\n"
            "find_package(OpenMP REQUIRED)\n"
            "set(GALA_AMD_ROOT \"\" CACHE PATH \"gala-gnn-acceleration-language_amd checkout\")\n"
            "set(GALA_REF_ROOT \"${CMAKE_CURRENT_SOURCE_DIR}/..\" CACHE PATH \"GALA reference root\")\n"
            "set_source_files_properties(gala.cu PROPERTIES LANGUAGE CXX)\n"
            "add_executable(gala_model gala.cu)\n"
            "target_compile_features(gala_model PRIVATE cxx_std_17)\n"
            "target_compile_options(gala_model PRIVATE -O2)\n"
            "target_compile_definitions(gala_model PRIVATE __HIP_PLATFORM_AMD__=1 USE_ROCM=1)\n"
            "target_include_directories(gala_model PRIVATE ${GALA_REF_ROOT} ${GALA_AMD_ROOT}/include /opt/rocm/include\n"
            "                           ${GALA_AMD_ROOT}/gala-gnn-acceleration-language_amd/host)\n"
            "target_link_directories(gala_model PRIVATE ${GALA_AMD_ROOT}/gala-gnn-acceleration-language_amd/gala)\n"
            "# torch's libraries first: one HIP runtime per process (torch's libamdhip64)\n"
            "target_link_libraries(gala_model PRIVATE \"${TORCH_LIBRARIES}\" gala_torch OpenMP::OpenMP_CXX)";
        cmakeCode.addCode(cm);
    }

    void initKernels(std::vector<CIRNode *> &program) override {
        std::string imports =
            "#include <torch/script.h>\n"
            "#include <torch/torch.h>\n"
            "#include <cmath>\n"
            "#include <cstdlib>\n"
            "#include <fstream>\n"
            "#include <iostream>\n"
            "#include <parallel/algorithm>\n"
            "#include <vector>\n"
            "#include <bits/stdc++.h>\n"
            "#include <omp.h>\n"
            "#include \"src/formats/csrc_matrix.h\"\n"
            "#include \"src/formats/dense_matrix.h\"\n"
            "#include \"src/ops/aggregators.h\"\n"
            "#include \"src/ops/tiling.h\"\n"
            "#include \"src/utils/mtx_io.h\"\n"
            "#include \"tests/common.h\"\n"
            "#include \"gala_torch.h\"\n";
        importCode.addCode(imports);

        std::string runtime =
            "// the program's device: GALA_DEVICE (\"cuda\" = the HIP device of PyTorch-ROCm, or \"cpu\")\n"
            "static torch::Device gala_program_device() {\n"
            "  const char *d = std::getenv(\"GALA_DEVICE\");\n"
            "  return torch::Device(d && *d ? d : \"cuda\");\n"
            "}\n"
            "static void gala_program_synchronize() {\n"
            "  if (gala_program_device().is_cuda()) torch::cuda::synchronize();\n"
            "}\n"
            "// GALA_DUMP=<file>: the first epoch's prediction and the initial weights (name, shape,\n"
            "// float32 values), for checking a generated program against another implementation\n"
            "template <class Net>\n"
            "static void gala_program_dump(size_t epoch, const torch::Tensor &prediction,\n"
            "                              const std::shared_ptr<Net> &net) {\n"
            "  const char *path = std::getenv(\"GALA_DUMP\");\n"
            "  if (!path || !*path || epoch != 1) return;\n"
            "  std::ofstream f(path, std::ios::binary);\n"
            "  auto put = [&](const std::string &name, torch::Tensor t) {\n"
            "    t = t.detach().to(torch::kCPU, torch::kFloat).contiguous();\n"
            "    f << name << '\\n' << t.dim();\n"
            "    for (auto s : t.sizes()) f << ' ' << s;\n"
            "    f << '\\n';\n"
            "    f.write(reinterpret_cast<const char *>(t.data_ptr<float>()), t.numel() * sizeof(float));\n"
            "  };\n"
            "  put(\"prediction\", prediction);\n"
            "  for (auto &p : net->named_parameters()) put(p.key(), p.value());\n"
            "}\n"
            "// ... and, appended after the first backward, the loss and every weight gradient\n"
            "template <class Net>\n"
            "static void gala_program_dump_grads(size_t epoch, const torch::Tensor &loss,\n"
            "                                    const std::shared_ptr<Net> &net) {\n"
            "  const char *path = std::getenv(\"GALA_DUMP\");\n"
            "  if (!path || !*path || epoch != 1) return;\n"
            "  std::ofstream f(path, std::ios::binary | std::ios::app);\n"
            "  auto put = [&](const std::string &name, torch::Tensor t) {\n"
            "    t = t.detach().to(torch::kCPU, torch::kFloat).contiguous();\n"
            "    f << name << '\\n' << t.dim();\n"
            "    for (auto s : t.sizes()) f << ' ' << s;\n"
            "    f << '\\n';\n"
            "    f.write(reinterpret_cast<const char *>(t.data_ptr<float>()), t.numel() * sizeof(float));\n"
            "  };\n"
            "  put(\"loss\", loss.reshape({1}));\n"
            "  for (auto &p : net->named_parameters())\n"
            "    if (p.value().grad().defined()) put(p.key() + \".grad\", p.value().grad());\n"
            "}\n"
            "// the reference runtime's names for the operator mirror's free functions\n"
            "using gala::edge_sddvv;\n"
            "using gala::edge_sddmm;\n"
            "using gala::gather_forward;\n"
            "using gala::node_spmv_backward_of_sddmm_nln;\n"
            "using gala::node_spmv_backward_of_sddmm_eaggr;\n"
            "using gala::inplace_softmax_sddvv;\n"
            "using gala::inplace_softmax_sddvv_mult;\n"
            "using gala::aggregate_edge_mul;\n"
            "using gala::aggregate_edge_mul_dir;\n";
        kernelCode.addCode(runtime);

        std::unordered_set<std::string> done;
        auto visit = [&](ComputeNode *c) {
            if (!c) return;
            const std::string name = getKernelName(c);
            if (done.insert(name).second) emitCall(c, name);
        };
        for (CIRNode *n : program) {
            if (auto *c = dynamic_cast<ComputeNode *>(n)) {
                visit(c);
            } else if (auto *loop = dynamic_cast<TrainingLoopNode *>(n)) {
                for (int i = 0; i < loop->getLoopNodeNum(); ++i) visit(loop->getNode(i));
            }
        }
    }

    // The features leave the program without requires_grad: CUDAGenerator creates them with
    // options_cu_float_grad (cuda.h:1381-1382), so every backward also formed and accumulated
    // d t_iden -- an [N, F] gradient nothing reads (5.7 GB per epoch at config 5's 11 M rows:
    // the first aggregation's backward, its ROW_BROADCAST and the accumulation, 7.7 ms).  The
    // weights' gradients are unchanged (checked bit for bit against the base spelling,
    // GALA_REFGEN_UNFUSED, which keeps it).
    void dataPrep(std::vector<CIRNode *> &program) override {
        std::string s =
            "  // GALA_SEED=<n>: torch's generators seeded before the model's weights are drawn (the\n"
            "  // reference seeds nothing: every run starts from other weights)\n"
            "  if (const char *seed = std::getenv(\"GALA_SEED\")) torch::manual_seed(std::atoll(seed));\n"
            "  torch::Device device = gala_program_device();\n"
            "  auto options_cu_int = torch::TensorOptions().dtype(torch::kInt).requires_grad(false).device(device);\n"
            "  auto options_cu_float_grad = torch::TensorOptions().dtype(torch::kFloat).requires_grad(true).device(device);\n"
            "  auto options_cu_float_ngrad = torch::TensorOptions().dtype(torch::kFloat).requires_grad(false).device(device);\n"
            "  auto options_cu_bool = torch::TensorOptions().dtype(torch::kBool).requires_grad(false).device(device);\n"
            "  auto options_cu_long = torch::TensorOptions().dtype(torch::kLong).device(device);\n"
            "  // features, labels and masks: host matrices copied into torch-owned device tensors\n"
            "  torch::Tensor t_iden = torch::from_blob(input_emb.vals_ptr(), {(int64_t)nrows, (int64_t)emb_size},\n"
            "                                         torch::kFloat).to(device).clone()" +
            std::string(std::getenv("GALA_REFGEN_UNFUSED") ? ".requires_grad_(true)" : "") + ";\n"
            "  torch::Tensor t_labs = torch::from_blob(labels.vals_ptr(), {(int64_t)nrows}, torch::kLong).to(device).clone();\n"
            "  torch::Tensor t_train_mask = torch::from_blob(train_mask.vals_ptr(), {(int64_t)nrows}, torch::kBool).to(device).clone();\n"
            "  torch::Tensor t_valid_mask = torch::from_blob(valid_mask.vals_ptr(), {(int64_t)nrows}, torch::kBool).to(device).clone();\n"
            "  torch::Tensor t_test_mask = torch::from_blob(test_mask.vals_ptr(), {(int64_t)nrows}, torch::kBool).to(device).clone();\n";
        preCode.addCode(s);
        std::unordered_set<std::string> seen;
        bool defaultLoaded = false;
        for (CIRNode *n : program) {
            if (auto *c = dynamic_cast<ComputeNode *>(n)) {
                transferInputs(c, seen, defaultLoaded);
            } else if (auto *loop = dynamic_cast<TrainingLoopNode *>(n)) {
                for (int i = 0; i < loop->getLoopNodeNum(); ++i) transferInputs(loop->getNode(i), seen, defaultLoaded);
            }
        }
    }

    // The base's writeCode (common.h:1722-1763) with the device retargeting and the dump hook.
    void writeCode(std::vector<CIRNode *> &program, std::vector<RelationEdge *> &dependencies,
                   std::vector<RelationEdge *> &associations, std::vector<TransformEdge *> &transforms) {
        (void)dependencies;
        (void)associations;
        initCMake();
        initKernels(program);
        commonPerCode();
        generateCode(program, transforms);
        for (Code *c : {&kernelCallCode, model.getDef(), model.getInit(), model.getForward(), &preCode,
                        model.getInv(), model.getPreCall(), model.getCall(), model.getPostCall(), &postCode})
            retarget(*c);
        denseOnMatrixCores(*model.getForward());
        denseOnMatrixCores(*model.getInv());
        if (!std::getenv("GALA_REFGEN_UNFUSED")) {   // (the unfused spelling: a bit-identity check)
            fuseGcnChains(*model.getForward());
            fuseGatChains(*model.getForward());
            trainRowsAndLoss(preCode, *model.getPostCall());
        }
        addDumpHook(*model.getPostCall());
        CodeGenerator::writeCode(cmakeCode, outStreamCMake);
        CodeGenerator::writeCode(importCode, outStreamModel);
        CodeGenerator::writeCode(kernelCode, outStreamModel);
        CodeGenerator::writeCode(kernelCallCode, outStreamModel);
        CodeGenerator::writeCode(*model.getDef(), outStreamModel);
        CodeGenerator::writeCode(*model.getInitCall(), outStreamModel, ", ", true, true);
        CodeGenerator::writeCode(*model.getInit(), outStreamModel);
        CodeGenerator::writeCode(*model.getForwardCallPre(), outStreamModel, "");
        CodeGenerator::writeCode(*model.getForwardCallInternal(), outStreamModel, "");
        CodeGenerator::writeCode(*model.getForwardCallPost(), outStreamModel);
        CodeGenerator::writeCode(*model.getForward(), outStreamModel);
        CodeGenerator::writeCode(preCode, outStreamModel);
        CodeGenerator::writeCode(*model.getInv(), outStreamModel);
        CodeGenerator::writeCode(*model.getPreCall(), outStreamModel, "");
        CodeGenerator::writeCode(*model.getCall(), outStreamModel, "");
        CodeGenerator::writeCode(*model.getPostCall(), outStreamModel);
        CodeGenerator::writeCode(postCode, outStreamModel);
        closeStream();
    }

private:
    // `<kernel name>_call(input_dense, offset_graph, columns_graph, value_graph[, bounds,
    // segments])`, the signature the base's autograd classes and direct calls use
    // (common.h:840-975, 1090-1127); its body is the mirror's aggregation with the node's
    // weighting and kernel sampling (cuda.h:172-205 decide the same three things).
    void emitCall(ComputeNode *c, const std::string &name) {
        const ComputeOp op = c->getOp();
        if (op != AGGREGATE_MUL_SUM_OP && op != AGGREGATE_MUL_SUM_DIRECT) return;  // others: `using` above
        DataInfo *g = c->getInput(1)->getDataInfo();
        const bool weighted = g->getWeighted();
        const bool tiled = hasDOpt(c->getInput(1), COL_TILE_DOPT);
        int nsamp = 0;
        for (auto &o : *c->getOpts())
            if (o.first == SAMPLE_COPT || o.first == SAMPLE_DYNAMIC_COPT) nsamp = (int)o.second;
        if (op == AGGREGATE_MUL_SUM_OP && nsamp == 0) plainAgg_.insert(name + "_AutoGrad");
        std::string fn = "torch::Tensor " + name +
                         "_call(torch::Tensor input_dense, torch::Tensor offset_graph, torch::Tensor columns_graph,\n"
                         "                     torch::Tensor value_graph";
        fn += tiled ? ", torch::Tensor bounds, int segments) {\n" : ") {\n  torch::Tensor bounds;\n  int segments = 1;\n";
        if (op == AGGREGATE_MUL_SUM_DIRECT) {
            fn += "  return gala::aggregate_node_mul_sum_direct_call(input_dense, offset_graph, columns_graph, value_graph,\n"
                  "                                                  bounds, segments, " + std::string(weighted ? "true" : "false") + ");\n}";
        } else {
            // kernel sampling reads the global (ra, rb) like the reference kernels (cuda.h:313-321)
            fn += "  return gala::aggregate_node_mul_sum_call(input_dense, offset_graph, columns_graph, value_graph, bounds,\n"
                  "                                           segments, " + std::string(weighted ? "true" : "false") + ", " +
                  std::to_string(nsamp) + ", " + (nsamp ? "global_ra, global_rb" : "5, 7") + ");\n}";
        }
        kernelCallCode.addCode(fn);
    }

    // One graph slot pair (forward 2g, backward 2g+1) as device tensors: the reference's
    // global_* vectors (what the base's autograd classes index) and the mirror's slots.
    // t: the tensor-name suffix ("0", "0_b"); idx: the graph index of its edge count nvals<idx>
    std::string slotCode(const std::string &t, const std::string &idx, const std::string &host, const std::string &seg,
                         bool tiled, bool weighted) {
        std::string s;
        if (tiled) {
            s += "  torch::Tensor t_offsets" + t + " = torch::from_blob(offset_ptr_" + host + ", {((int64_t)nrows + 1) * " + seg +
                 "}, torch::kInt).to(device).clone();\n"
                 "  torch::Tensor t_cols" + t + " = torch::from_blob(col_ptr_" + host + ", {(int64_t)nvals" + idx +
                 "}, torch::kInt).to(device).clone();\n"
                 "  torch::Tensor t_vals" + t + " = torch::from_blob(val_ptr_" + host + ", {(int64_t)nvals" + idx +
                 "}, torch::kFloat).to(device).clone();\n";
        } else {
            s += "  torch::Tensor t_offsets" + t + " = torch::from_blob(" + host + ".offset_ptr(), {(int64_t)nrows + 1}, "
                 "torch::kInt).to(device).clone();\n"
                 "  torch::Tensor t_cols" + t + " = torch::from_blob(" + host + ".ids_ptr(), {(int64_t)nvals" + idx +
                 "}, torch::kInt).to(device).clone();\n"
                 "  torch::Tensor t_vals" + t + " = torch::from_blob(" + host + ".vals_ptr(), {(int64_t)nvals" + idx +
                 "}, torch::kFloat).to(device).clone();\n";
        }
        s += "  global_offset_graph.push_back(t_offsets" + t + ");\n"
             "  global_columns_graph.push_back(t_cols" + t + ");\n"
             "  global_value_graph.push_back(t_vals" + t + ");\n";
        s += register_(t, tiled, weighted, host, seg);
        return s;
    }

    // the mirror's slot registry: a one-segment graph's hub-row plan; a column-tiled graph
    // (the base's total_bounds_<name> / segments_<name>, common.h:1365-1402) gets its merged
    // rows, on which its unweighted SpMMs run as one segment
    static std::string register_(const std::string &t, bool tiled, bool weighted, const std::string &host,
                                 const std::string &seg) {
        const std::string b = tiled ? "total_bounds_" + host + ", " + seg : "torch::Tensor(), 1";
        return "  gala::global_slots().push(t_offsets" + t + ", t_cols" + t + ", t_vals" + t + ", " + b + ", " +
               (weighted ? "true" : "false") + ");\n";
    }

    std::string graphPair(DataNode *d, const std::string &name, int index, bool directed, bool weighted) {
        const std::string idx = std::to_string(index);
        const bool tiled = hasDOpt(d, COL_TILE_DOPT);
        std::string s = slotCode(idx, idx, tiled ? name : "adj" + idx, "segments_" + name, tiled, weighted);
        if (!directed) {  // undirected: slot 2g+1 is the same tensors (cuda.h:1253-1257)
            s += "  global_offset_graph.push_back(t_offsets" + idx + ");\n"
                 "  global_columns_graph.push_back(t_cols" + idx + ");\n"
                 "  global_value_graph.push_back(t_vals" + idx + ");\n";
            s += register_(idx, tiled, weighted, tiled ? name : "adj" + idx, "segments_" + name);
        } else {          // directed: the transposed graph the host code built (adj<g>_b)
            s += slotCode(idx + "_b", idx, tiled ? name + "_b" : "adj" + idx + "_b", "segments_" + name + "_b", tiled,
                          weighted);
        }
        return s;
    }

    // The graph inputs of one compute node, each transferred once (the order and slot
    // numbering of cuda.h:1051-1305: the default graph first, then every other CSR input)
    void transferInputs(ComputeNode *c, std::unordered_set<std::string> &seen, bool &defaultLoaded) {
        if (!c) return;
        std::string code;
        for (int i = 0; i < c->getNumInputs(); ++i) {
            DataNode *d = c->getInput(i);
            DataInfo *info = d->getDataInfo();
            if (!defaultLoaded && info->getIndex() > 0) {
                const std::string name = info->getDefaultName().empty() ? d->getName() : info->getDefaultName();
                if (!seen.count(name) && info->getFormat() == CSR_STYPE) {
                    defaultLoaded = true;
                    seen.insert(name);
                    code += graphPair(d, name, info->getDefaultIndex(), info->getDefaultDirected(), info->getWeighted());
                }
            }
            if (seen.count(d->getName())) continue;
            if (info->getFormat() != CSR_STYPE || info->getDerived()) continue;
            int index = (int)seen.size();
            if (info->getIndex() != -1) index = info->getIndex();
            seen.insert(d->getName());
            if (d->getName() == "attn" || d->getName() == "val") continue;  // edge values, not graphs
            info->setIndex(index);
            code += graphPair(d, d->getName(), index, info->getDirected(), info->getWeighted());
        }
        if (!code.empty()) preCode.addCode(code);
    }

    static void replaceAll(std::string &s, const std::string &from, const std::string &to) {
        for (size_t p = s.find(from); p != std::string::npos; p = s.find(from, p + to.size())) s.replace(p, from.size(), to);
    }

    // the base generator's device-specific spellings, on the program's device
    static void retarget(Code &code) {
        for (int i = 0; i < code.getNum(); ++i) {
            std::string *l = code.atLine(i);
            replaceAll(*l, ".device(torch::kCUDA, 0)", ".device(gala_program_device())");
            replaceAll(*l, "cudaDeviceSynchronize();", "gala_program_synchronize();");
        }
    }

    // The model's hidden Linear layers (`fcN->forward(x)`, SAGE's `sfcN->forward(x)`,
    // common.h:1205-1280) as the mirror's FFN op over the same parameters: the forward is
    // at::linear's (at::addmm, or the matrix-core kernel for 33..64 outputs) and the weight /
    // bias gradients run on gala_dense_grad_f32, split over rows.  torch::nn::Linear's
    // backward takes dW = dYᵀX as one library GEMM whose only parallelism is the 128x128
    // output (K = the 11 M rows of config 5: 12.0 ms per call on MI355X, 5.0 ms here;
    // profiles/r04_refgen_config5_kernels.txt).
    // The attention Linears (`efcN->forward(x)`, Linear(hs, 1): attnL / attnR of the GAT
    // layer, common.h:1248-1260) run as the mirror's head-attention op with one head over the
    // same parameters (gala_head_attn_f32 / _bwd_f32, the weight gradient on
    // gala_dense_grad_f32): torch's Linear(32, 1) forward is a hipBLASLt GEMM with a 32 x 1
    // tile, 2.2 ms per call at 2.4 M rows for 313 MB read (profiles/
    // r05_refgen_gat_products_kernels.csv), and its backward three more such GEMMs.  The
    // attention logits are the same dot products summed in another order (the reference's
    // BLAS order is not pinned either).
    static void denseOnMatrixCores(Code &code) {
        for (int i = 0; i < code.getNum(); ++i) {
            std::string *l = code.atLine(i);
            for (const std::string pre : {"efc", "sfc", "fc"}) {
                for (size_t p = l->find(pre); p != std::string::npos; p = l->find(pre, p + 1)) {
                    if (p > 0 && (std::isalnum((unsigned char)(*l)[p - 1]) || (*l)[p - 1] == '_')) continue;
                    size_t q = p + pre.size();
                    while (q < l->size() && std::isdigit((unsigned char)(*l)[q])) ++q;
                    const std::string call = "->forward(";
                    if (q == p + pre.size() || l->compare(q, call.size(), call) != 0) continue;
                    const std::string mod = l->substr(p, q - p);
                    size_t a = q + call.size(), e = a;
                    for (int depth = 1; e < l->size(); ++e) {
                        if ((*l)[e] == '(') ++depth;
                        if ((*l)[e] == ')' && --depth == 0) break;
                    }
                    if (e >= l->size()) continue;
                    const std::string arg = l->substr(a, e - a);
                    const std::string fn = pre == "efc" ? "gala::head_attn_apply(" : "gala::ffn_apply(";
                    l->replace(p, e + 1 - p, fn + arg + ", " + mod + "->weight, " + mod + "->bias)");
                }
            }
        }
    }

    // The base emits a GCN layer as torch ops around the aggregation's autograd class:
    // `res = norm * x;` (ROW_BROADCAST), `res = torch::relu(res);`, the aggregation (an
    // `if (ep % mod_v == 0)` pair of identical apply calls), `res = norm * res;`
    // (common.h:928-978, 1150-1184).  On config 5's 11 M rows each such torch op is a 5.7 GB
    // pass (a ROW_BROADCAST 1.8 ms, a ReLU 2.9 ms, forward and backward alike).  A chain
    //     [res = act * X;] [res = torch::relu(res);] [res = pre * res;] AGG [res = post * res;]
    // around an unsampled aggregation becomes the mirror's fused op over the same slot,
    //     res = gala::gcn_aggregate_relu_apply(X, act, pre, post, li);   (or gcn_aggregate_apply)
    // whose forward and backward are the unfused chain's roundings bit for bit (the ROW_
    // BROADCASTs in the aggregation's prologue / epilogue, relu as torch's GPU kernel).
    // Statements of any other shape are left as they are.
    struct FwdStmt {
        enum Kind { Other, Mul, Relu, Agg, AttnAgg, EdgeSum, LeakyDecl, Leaky, Softmax, HeadAttn } kind = Other;
        // Mul: a = scale, b = source; Agg: a = class, b = slot index; AttnAgg: a = class,
        // b = slot, c = source; EdgeSum: a = attn_l, b = attn_r, c = slot; LeakyDecl: a = slope;
        // Softmax: b = slot; HeadAttn: lhs = gala::head_attn_apply(a, c->weight, c->bias), b = lhs
        std::string text, a, b, c;
    };

    static std::vector<FwdStmt> splitForward(const std::string &t) {
        static const std::regex mul("^res = (\\w+) \\* (\\w+);$"), relu("^res = torch::relu\\(res\\);$"),
            app("^res = (\\w+)::apply\\(res, (\\d+)\\);$"),
            app_attn("^res = (\\w+)::apply\\((\\w+), attn, (\\d+)\\);$"),
            edge("^attn = aggregate_edge_sum_AutoGrad::apply\\((\\w+), (\\w+), (\\d+)\\);$"),
            leaky_decl("^torch::nn::LeakyReLU leaky_relu\\(torch::nn::LeakyReLUOptions\\(\\)\\.negative_slope\\(([0-9.eE+-]+)\\)\\);$"),
            leaky("^attn = leaky_relu->forward\\(attn\\);$"),
            softmax("^attn = non_lnr_op_softmax_AutoGrad::apply\\(attn, (\\d+)\\);$"),
            head_attn("^(\\w+) = gala::head_attn_apply\\((\\w+), (\\w+)->weight, \\3->bias\\);$");
        std::vector<FwdStmt> out;
        size_t p = 0;
        auto trim = [](std::string x) {
            const size_t a = x.find_first_not_of(" \t\n"), b = x.find_last_not_of(" \t\n");
            return a == std::string::npos ? std::string() : x.substr(a, b - a + 1);
        };
        auto block = [&](size_t open, size_t &close) {  // body of the {...} opening at `open`
            int depth = 0;
            for (size_t i = open; i < t.size(); ++i) {
                if (t[i] == '{') ++depth;
                if (t[i] == '}' && --depth == 0) {
                    close = i;
                    return trim(t.substr(open + 1, i - open - 1));
                }
            }
            close = std::string::npos;
            return std::string();
        };
        const std::string ifkey = "if (ep % mod_v == 0)";
        while (p < t.size()) {
            const size_t q = t.find_first_not_of(" \t\n", p);
            if (q == std::string::npos) {
                out.push_back({FwdStmt::Other, t.substr(p), "", ""});
                break;
            }
            FwdStmt st;
            if (t.compare(q, ifkey.size(), ifkey) == 0) {
                size_t c1 = std::string::npos, c2 = std::string::npos;
                const size_t o1 = t.find('{', q);
                const std::string b1 = o1 == std::string::npos ? "" : block(o1, c1);
                const size_t e = c1 == std::string::npos ? c1 : t.find_first_not_of(" \t\n", c1 + 1);
                const bool has_else = e != std::string::npos && t.compare(e, 4, "else") == 0;
                const size_t o2 = has_else ? t.find('{', e) : std::string::npos;
                const std::string b2 = o2 == std::string::npos ? "" : block(o2, c2);
                std::smatch m1, m2;
                if (c2 != std::string::npos && std::regex_match(b1, m1, app) && std::regex_match(b2, m2, app) &&
                    m1[0] == m2[0]) {
                    st = {FwdStmt::Agg, t.substr(p, c2 + 1 - p), m1[1], m1[2], ""};
                    out.push_back(st);
                    p = c2 + 1;
                    continue;
                }
                if (c2 != std::string::npos && std::regex_match(b1, m1, app_attn) &&
                    std::regex_match(b2, m2, app_attn) && m1[0] == m2[0]) {
                    st = {FwdStmt::AttnAgg, t.substr(p, c2 + 1 - p), m1[1], m1[3], m1[2]};
                    out.push_back(st);
                    p = c2 + 1;
                    continue;
                }
            }
            const size_t semi = t.find(';', q);
            const size_t end = semi == std::string::npos ? t.size() : semi + 1;
            st.text = t.substr(p, end - p);
            const std::string body = trim(st.text);
            std::smatch m;
            if (std::regex_match(body, m, mul)) st = {FwdStmt::Mul, st.text, m[1], m[2], ""};
            else if (std::regex_match(body, relu)) st = {FwdStmt::Relu, st.text, "", "", ""};
            else if (std::regex_match(body, m, edge)) st = {FwdStmt::EdgeSum, st.text, m[1], m[2], m[3]};
            else if (std::regex_match(body, m, leaky_decl)) st = {FwdStmt::LeakyDecl, st.text, m[1], "", ""};
            else if (std::regex_match(body, leaky)) st = {FwdStmt::Leaky, st.text, "", "", ""};
            else if (std::regex_match(body, m, softmax)) st = {FwdStmt::Softmax, st.text, "", m[1], ""};
            else if (std::regex_match(body, m, head_attn)) st = {FwdStmt::HeadAttn, st.text, m[2], m[1], m[3]};
            out.push_back(st);
            p = end;
        }
        return out;
    }

    void fuseGcnChains(Code &fwd) {
        std::string t;
        for (int i = 0; i < fwd.getNum(); ++i) t += *fwd.atLine(i) + "\n";
        std::vector<FwdStmt> st = splitForward(t);
        std::string out;
        size_t done = 0;  // statements [0, done) are emitted
        for (size_t k = 0; k < st.size(); ++k) {
            if (st[k].kind != FwdStmt::Agg || !plainAgg_.count(st[k].a)) continue;
            // prologue, walking back: [Mul(act, X)] [Relu] [Mul(pre, res | X)]
            size_t j = k;
            std::string X = "res", act, pre, post;
            bool relu = false;
            if (j > done && st[j - 1].kind == FwdStmt::Mul) {
                pre = st[j - 1].a;
                X = st[j - 1].b;
                --j;
            }
            if (X == "res" && j > done && st[j - 1].kind == FwdStmt::Relu) {
                relu = true;
                --j;
                if (j > done && st[j - 1].kind == FwdStmt::Mul) {
                    act = st[j - 1].a;
                    X = st[j - 1].b;
                    --j;
                }
            }
            size_t last = k;   // epilogue: Mul(post, res)
            if (k + 1 < st.size() && st[k + 1].kind == FwdStmt::Mul && st[k + 1].b == "res") {
                post = st[k + 1].a;
                last = k + 1;
            }
            if (!relu && pre.empty() && post.empty()) continue;   // nothing to fuse: as emitted
            for (size_t i = done; i < j; ++i) out += st[i].text;
            const std::string none = "torch::Tensor()";
            auto arg = [&](const std::string &v) { return v.empty() ? none : v; };
            out += "\n        // ROW_BROADCAST / RELU / AGGREGATE / ROW_BROADCAST fused (HIPGenerator)\n";
            if (relu)
                out += "        res = gala::gcn_aggregate_relu_apply(" + X + ", " + arg(act) + ", " + arg(pre) + ", " +
                       arg(post) + ", " + st[k].b + ");";
            else
                out += "        res = gala::gcn_aggregate_apply(" + X + ", " + arg(pre) + ", " + arg(post) + ", " +
                       st[k].b + ");";
            done = last + 1;
            k = last;
        }
        for (size_t i = done; i < st.size(); ++i) out += st[i].text;
        *fwd.atLine(0) = out;
        for (int i = 1; i < fwd.getNum(); ++i) fwd.atLine(i)->clear();
    }

    // The base emits a GAT layer (common.h:622-894, 1175-1184) as four steps over E-long
    // edge tensors: the edge sum's autograd class (K5), torch's LeakyReLU, the softmax class
    // (torch exp / clamp / reciprocal around K7 and K8) and the attention-weighted aggregation
    // class -- with their backwards (K9, the softmax backward's torch ops around K7 / K8, K7 for
    // the logits' gradient): on the Products shape 30.8 ms per epoch where galac's fused layer
    // takes 20.8 (profiles/r05_refgen_gat_products.jsonl).  The chain
    //     attn = aggregate_edge_sum_AutoGrad::apply(L, R, li);  [LeakyReLU declaration]
    //     attn = leaky_relu->forward(attn);  attn = non_lnr_op_softmax_AutoGrad::apply(attn, li);
    //     AGG(X, attn, li)   (the `if (ep % mod_v == 0)` pair)
    // becomes the mirror's fused layer over the same slot in REF mode,
    //     res = gala::gat_aggregate_apply(L, R, X, li, slope, GALA_SOFTMAX_REF);
    // (the same chain of operations per edge, one pass per row; alpha = p * q with the
    // reference's clamp, 1e-12 and sequential row sums; gradients d aL = d aR = the row sums of
    // the LeakyReLU'd softmax gradient, as the base's classes return them).  When R is
    // `gala::head_attn_apply(X, W->weight, W->bias)` of the aggregated rows themselves, the
    // layer recomputes it from the rows it gathers (gat_aggregate_ffn_apply, galac's spelling)
    // and the statement goes when nothing else reads R.  The values are the chain's within
    // fp32 rounding, not bit for bit: the fused kernels sum in the chain's order but round
    // alpha = p * q once per edge where the chain stores it (tests/test_gpu_refgen.py checks
    // the program against galac's IR in float64 at 1e-4; GALA_REFGEN_UNFUSED keeps the base's
    // spelling).
    void fuseGatChains(Code &fwd) {
        std::string t;
        for (int i = 0; i < fwd.getNum(); ++i) t += *fwd.atLine(i) + "\n";
        std::vector<FwdStmt> st = splitForward(t);
        static const std::regex word_attn("\\battn\\b");
        auto mentions = [](const std::string &text, const std::string &name) {
            return std::regex_search(text, std::regex("\\b" + name + "\\b"));
        };
        std::vector<bool> drop(st.size(), false);
        std::vector<std::string> repl(st.size());
        std::string slope = "0.2";
        bool any = false;
        for (size_t k = 0; k < st.size(); ++k) {
            if (st[k].kind == FwdStmt::LeakyDecl) slope = st[k].a;
            if (st[k].kind != FwdStmt::AttnAgg || !plainAgg_.count(st[k].a) || k < 3) continue;
            const std::string li = st[k].b, X = st[k].c;
            if (st[k - 1].kind != FwdStmt::Softmax || st[k - 1].b != li || st[k - 2].kind != FwdStmt::Leaky) continue;
            size_t e = k - 3;
            if (st[e].kind == FwdStmt::LeakyDecl) {   // kept: later layers use the variable
                if (e == 0) continue;
                --e;
            }
            if (st[e].kind != FwdStmt::EdgeSum || st[e].c != li) continue;
            // `attn` must not be read after the chain before it is assigned again
            bool attn_dead = true;
            for (size_t i = k + 1; i < st.size(); ++i) {
                if (!std::regex_search(st[i].text, word_attn)) continue;
                attn_dead = st[i].kind == FwdStmt::EdgeSum;
                break;
            }
            if (!attn_dead) continue;
            const std::string L = st[e].a, R = st[e].b;
            // R = head_attn_apply(X, W->weight, W->bias) just before, with only other attention
            // Linears (not assigning X) in between
            long h = -1;
            for (long i = (long)e - 1; i >= 0; --i) {
                if (st[i].kind != FwdStmt::HeadAttn || st[i].b == X) break;
                if (st[i].b == R) {
                    if (st[i].a == X) h = i;
                    break;
                }
            }
            std::string rest;
            for (size_t i = k + 1; i < st.size(); ++i) rest += st[i].text;
            std::string call;
            if (h >= 0 && R != L) {
                const std::string W = st[h].c;
                call = "res = gala::gat_aggregate_ffn_apply(" + L + ", " + X + ", " + W + "->weight, " + W + "->bias, " +
                       li + ", " + slope + ", GALA_SOFTMAX_REF);";
                if (!mentions(rest, R)) drop[h] = true;
            } else {
                call = "res = gala::gat_aggregate_apply(" + L + ", " + R + ", " + X + ", " + li + ", " + slope +
                       ", GALA_SOFTMAX_REF);";
            }
            repl[e] = "\n        // EDGE SUM / LEAKY RELU / SOFTMAX / AGGREGATE fused (HIPGenerator)\n        " + call;
            drop[k - 2] = drop[k - 1] = drop[k] = true;
            any = true;
        }
        if (!any) return;
        std::string out;
        for (size_t i = 0; i < st.size(); ++i) {
            if (!repl[i].empty()) out += repl[i];
            else if (!drop[i]) out += st[i].text;
        }
        *fwd.atLine(0) = out;
        for (int i = 1; i < fwd.getNum(); ++i) fwd.atLine(i)->clear();
    }

    // The training loop's loss (common.h:1506-1560): the training rows by index_select over
    // the mask's row list (computed once) instead of boolean indexing -- the same rows in the
    // same order, and the backward scatters one gradient per row either way -- and the
    // CrossEntropyLoss (mean) as log_softmax + gather + mean: the same prediction and
    // gradients bit for bit (d loss / d pred = -1/n at the label, then log_softmax's
    // backward); the loss value is the same sum taken in another order.  torch's
    // nll_loss_forward_reduce kernel reduces in one workgroup: 7.9 ms per epoch at config 5's
    // 3.3 M training rows (profiles/r04_refgen_config5_kernels.txt), its backward 5.4 ms.
    void trainRowsAndLoss(Code &pre, Code &post) {
        bool used = false;
        for (int i = 0; i < post.getNum(); ++i) {
            std::string *l = post.atLine(i);
            const size_t n0 = l->size();
            replaceAll(*l, "prediction.index({t_train_mask})", "prediction.index_select(0, gala_train_rows)");
            replaceAll(*l, "t_labs.index({t_train_mask})", "t_labs.index_select(0, gala_train_rows)");
            replaceAll(*l, "auto criterion = torch::nn::CrossEntropyLoss();", "");
            replaceAll(*l, "criterion(prediction_train, labels_train)", "gala_cross_entropy(prediction_train, labels_train)");
            used = used || l->size() != n0 || l->find("gala_train_rows") != std::string::npos;
        }
        if (!used) return;
        std::string rows = "  // the training rows, once (the loop's index_select)\n"
                           "  torch::Tensor gala_train_rows = t_train_mask.nonzero().reshape({-1});\n";
        pre.addCode(rows);
        std::string ce = "// CrossEntropyLoss (mean) as log_softmax + gather + mean\n"
                         "static torch::Tensor gala_cross_entropy(const torch::Tensor &pred, const torch::Tensor &labels) {\n"
                         "  return -torch::log_softmax(pred, 1).gather(1, labels.reshape({-1, 1})).mean();\n"
                         "}";
        kernelCode.addCode(ce);
    }

    std::unordered_set<std::string> plainAgg_;   // autograd classes of unsampled aggregations

    // after the loop's `prediction = net->forward(...)[0];`, and before its first
    // `optimizer.step();` (common.h:1506-1560)
    static void addDumpHook(Code &post) {
        bool fwd = false, grads = false;
        for (int i = 0; i < post.getNum(); ++i) {
            std::string *l = post.atLine(i);
            const std::string key = "mod_v)[0];\n", step = "    optimizer.step();";
            size_t p = l->find(key);
            if (!fwd && p != std::string::npos) {
                l->insert(p + key.size(), "    gala_program_dump(epoch, prediction, net);\n");
                fwd = true;
            }
            p = l->find(step);
            if (!grads && p != std::string::npos) {
                l->insert(p, "    gala_program_dump_grads(epoch, d_loss, net);\n");
                grads = true;
            }
        }
    }
};

#endif  // GALA_HIP_CODEGEN_H

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
#include <iostream>
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
        std::unordered_set<int> slots;
        bool defaultLoaded = false;
        for (CIRNode *n : program) {
            if (auto *c = dynamic_cast<ComputeNode *>(n)) {
                transferInputs(c, seen, slots, defaultLoaded);
            } else if (auto *loop = dynamic_cast<TrainingLoopNode *>(n)) {
                for (int i = 0; i < loop->getLoopNodeNum(); ++i) transferInputs(loop->getNode(i), seen, slots, defaultLoaded);
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
        const State before = save();
        generateCode(program, transforms);
        const State after = save();
        load(before);   // the dry run: which forward entries each in-loop node emitted
        const std::vector<Span> spans = forwardSpans(program, transforms);
        Code dry = *model.getForward();
        load(after);
        Code &fwd = *model.getForward();
        bool same = dry.getNum() <= fwd.getNum();
        for (int i = 0; same && i < dry.getNum(); ++i) same = *dry.atLine(i) == *fwd.atLine(i);
        if (!same) {
            std::cerr << "HIPGenerator: the dry run's forward differs from generateCode's; no fusion is safe\n";
            std::exit(3);
        }
        for (Code *c : {&kernelCallCode, model.getDef(), model.getInit(), model.getForward(), &preCode,
                        model.getInv(), model.getPreCall(), model.getCall(), model.getPostCall(), &postCode})
            retarget(*c);
        denseOnMatrixCores(*model.getForward());
        denseOnMatrixCores(*model.getInv());
        if (!std::getenv("GALA_REFGEN_UNFUSED")) {   // (the unfused spelling: a bit-identity check)
            fuseGcnChains(fwd, spans);
            fuseGatChains(fwd, spans);
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
    // numbering of cuda.h:1051-1305: the default graph first, then every other CSR input).
    // Each graph index is transferred once: under gala_train's training subgraph
    // (middle-end.h:39-210) an untiled program meets its loaded graph twice -- as the
    // subgraphs' default graph "adj" (index 0) and by its own name adj0 -- and cuda.h emits
    // dA_csrOffsets0 both times (a redeclaration nvcc would refuse); here the second is skipped.
    void transferInputs(ComputeNode *c, std::unordered_set<std::string> &seen, std::unordered_set<int> &slots,
                        bool &defaultLoaded) {
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
                    if (slots.insert(info->getDefaultIndex()).second)
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
            if (slots.insert(index).second)
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

    // ---- fusions, recognised on the CIR -------------------------------------------------
    // The base emits each in-loop node's statements into the forward (one Code entry per
    // statement) from the node's op, operand names and slot indices (common.h:511-1377).  The
    // fusions below recognise node chains on those same fields -- ops, names (the emitted
    // program's data flow is by name), graph indices, compute options -- and replace exactly
    // the forward entries the chain's nodes emitted.  Which entries a node emitted comes from a
    // dry run of the base's own generateOpCode over the program (forwardSpans), checked entry
    // for entry against the forward generateCode wrote; a mismatch stops the generator rather
    // than leaving a fusion silently off.

    // The sections generateCode writes into, saved and restored around the dry run.
    struct State {
        Code cmake, imports, kernels, kernelCalls, autoGrad, pre, post;
        Model model;
        std::vector<std::string> functions;
    };
    State save() const {
        State s;
        s.cmake = cmakeCode;
        s.imports = importCode;
        s.kernels = kernelCode;
        s.kernelCalls = kernelCallCode;
        s.autoGrad = autoGradCode;
        s.pre = preCode;
        s.post = postCode;
        s.model = model;
        s.functions = generatedFunctions;
        return s;
    }
    void load(const State &s) {
        cmakeCode = s.cmake;
        importCode = s.imports;
        kernelCode = s.kernels;
        kernelCallCode = s.kernelCalls;
        autoGradCode = s.autoGrad;
        preCode = s.pre;
        postCode = s.post;
        model = s.model;
        generatedFunctions = s.functions;
    }

    // One in-loop node and the forward entries [first, last) it emitted.
    struct Span {
        ComputeNode *node;
        int first, last;
        bool edgeUpdate;   // the base's hasFFNEdgeUpdate when the node was emitted (attention aggregation form)
        int fcEdge;        // its fcEdgeCount then (an FFN_OP_EDGE's module is efc<fcEdge>)
    };

    // generateCode's node walk (common.h:1378-1442) with the base's generateOpCode, recording
    // each in-loop node's forward entries.  Run on the state generateCode started from.
    std::vector<Span> forwardSpans(std::vector<CIRNode *> &program, std::vector<TransformEdge *> &transforms) {
        std::vector<int> inputSizes;
        int fcCount = 0, fcEdgeCount = 0, fcSelfCount = 0, epCount = 0;
        bool hasFFNEdgeUpdate = false, hasEdgeMulAggr = false;
        std::unordered_set<std::string> autograds;
        std::vector<Span> spans;
        for (CIRNode *n : program) {
            if (auto *c = dynamic_cast<ComputeNode *>(n)) {
                generateOpCode(c, fcCount, fcEdgeCount, fcSelfCount, epCount, true, hasFFNEdgeUpdate, hasEdgeMulAggr,
                               autograds, inputSizes, transforms);
                continue;
            }
            auto *loop = dynamic_cast<TrainingLoopNode *>(n);
            for (int i = 0; loop && i < loop->getLoopNodeNum(); ++i) {
                auto *c = dynamic_cast<ComputeNode *>(loop->getNode(i));
                Span s{c, model.getForward()->getNum(), 0, hasFFNEdgeUpdate, fcEdgeCount};
                generateOpCode(c, fcCount, fcEdgeCount, fcSelfCount, epCount, false, hasFFNEdgeUpdate, hasEdgeMulAggr,
                               autograds, inputSizes, transforms);
                s.last = model.getForward()->getNum();
                spans.push_back(s);
            }
        }
        return spans;
    }

    // the value a node's statement assigns, and its operand names, as the base spells them
    std::string out(const Span &s) { return generateOutputString(s.node, false); }
    static std::string in(const Span &s, int i) { return s.node->getInput(i)->getName(); }
    static ComputeOp opOf(const Span &s) { return s.node->getOp(); }
    static bool sampled(ComputeNode *c) {
        for (auto &o : *c->getOpts())
            if (o.first == SAMPLE_COPT || o.first == SAMPLE_DYNAMIC_COPT) return true;
        return false;
    }
    // the slot an in-loop aggregation's autograd call takes: 0 on validation epochs, its graph's
    // index otherwise (common.h:1003-1010; the index is a training subgraph's under gala_train)
    static std::string slotExpr(int idx) {
        return idx == 0 ? std::string("0") : "ep % mod_v == 0 ? 0 : " + std::to_string(idx);
    }
    // Is `name` still read after span `upto`?  Judged on the statements the forward holds
    // after it (the base spells some operands independently of the node's inputs, e.g.
    // FFN_OP_SELF's `res`): the first later statement that mentions the name must assign it
    // without reading it, otherwise the value is live.
    static bool mentions(const std::string &t, const std::string &name) {
        auto ident = [](char c) { return std::isalnum((unsigned char)c) || c == '_'; };
        for (size_t p = t.find(name); p != std::string::npos; p = t.find(name, p + 1))
            if ((p == 0 || !ident(t[p - 1])) && (p + name.size() >= t.size() || !ident(t[p + name.size()]))) return true;
        return false;
    }
    static bool readLater(Code &fwd, const std::vector<Span> &sp, size_t upto, const std::string &name) {
        for (int e = sp[upto].last; e < fwd.getNum(); ++e) {
            const std::string &t = *fwd.atLine(e);
            if (!mentions(t, name)) continue;
            const size_t a = t.find_first_not_of(" \t\n");
            const std::string lhs = name + " = ";
            if (a == std::string::npos || t.compare(a, lhs.size(), lhs) != 0) return true;
            return mentions(t.substr(a + lhs.size()), name) || t.find(';', a) + 1 < t.size();
        }
        return false;
    }
    // the forward entries of spans [a, b] replaced by one statement
    static void replaceSpans(Code &fwd, const std::vector<Span> &sp, size_t a, size_t b, const std::string &stmt) {
        for (size_t i = a; i <= b; ++i)
            for (int e = sp[i].first; e < sp[i].last; ++e) fwd.atLine(e)->clear();
        *fwd.atLine(sp[a].first) = stmt;
    }

    // The base emits a GCN layer as torch ops around the aggregation's autograd class: ROW_
    // BROADCAST `res = norm * x;`, NON_LINEARITY `res = torch::relu(res);`, the aggregation (an
    // `if (ep % mod_v == 0)` pair of apply calls) and the ROW_BROADCAST after it
    // (common.h:1003-1010, 1150-1184).  On config 5's 11 M rows each such torch op is a 5.7 GB
    // pass (a ROW_BROADCAST 1.8 ms, a ReLU 2.9 ms, forward and backward alike).  A node chain
    //     [ROW_BROADCAST(act, X)] [RELU] [ROW_BROADCAST(pre, .)] AGGREGATE_MUL_SUM [ROW_BROADCAST(post, .)]
    // around an unsampled, unweighted aggregation (each node reading the previous one's
    // value, the intermediate values read by nothing after the chain) becomes the mirror's
    // fused op over the same slot,
    //     res = gala::gcn_aggregate_relu_apply(X, act, pre, post, li);   (or gcn_aggregate_apply)
    // whose forward and backward are the unfused chain's roundings bit for bit (the ROW_
    // BROADCASTs in the aggregation's prologue / epilogue, relu as torch's GPU kernel).  li
    // keeps the base's choice of slot per epoch (a training subgraph's off validation epochs).
    void fuseGcnChains(Code &fwd, const std::vector<Span> &sp) {
        size_t done = 0;   // spans [0, done) are taken
        for (size_t k = 0; k < sp.size(); ++k) {
            const Span &ag = sp[k];
            if (opOf(ag) != AGGREGATE_MUL_SUM_OP || ag.edgeUpdate || sampled(ag.node) || ag.last == ag.first) continue;
            // the longest chain first; a ReLU whose output is still read later stays unfused
            for (bool withRelu : {true, false}) {
                size_t j = k;
                std::string X = in(ag, 0), act, pre, post;
                bool relu = false;
                std::vector<std::string> inner;   // values the chain writes before its last node
                if (j > done && opOf(sp[j - 1]) == ROW_BROADCAST_OP && out(sp[j - 1]) == X) {
                    pre = in(sp[j - 1], 0);
                    inner.push_back(X);
                    X = in(sp[j - 1], 1);
                    --j;
                }
                if (withRelu && j > done && opOf(sp[j - 1]) == NON_LNR_OP_RELU && out(sp[j - 1]) == X) {
                    relu = true;
                    inner.push_back(X);
                    X = in(sp[j - 1], 0);
                    --j;
                    if (j > done && opOf(sp[j - 1]) == ROW_BROADCAST_OP && out(sp[j - 1]) == X) {
                        act = in(sp[j - 1], 0);
                        inner.push_back(X);
                        X = in(sp[j - 1], 1);
                        --j;
                    }
                }
                size_t last = k;
                if (k + 1 < sp.size() && opOf(sp[k + 1]) == ROW_BROADCAST_OP && in(sp[k + 1], 1) == out(ag)) {
                    post = in(sp[k + 1], 0);
                    inner.push_back(out(ag));
                    last = k + 1;
                }
                if (!relu && pre.empty() && post.empty()) break;   // nothing to fuse: as emitted
                const std::string res = out(sp[last]);
                bool dead = true;
                for (const std::string &v : inner)
                    dead = dead && (v == res || !readLater(fwd, sp, last, v));
                if (!dead) continue;
                const int idx = ag.node->getInput(1)->getDataInfo()->getIndex();
                auto arg = [](const std::string &v) { return v.empty() ? std::string("torch::Tensor()") : v; };
                std::string stmt = "\n        // ROW_BROADCAST / RELU / AGGREGATE / ROW_BROADCAST fused (HIPGenerator)\n        " + res;
                if (relu)
                    stmt += " = gala::gcn_aggregate_relu_apply(" + X + ", " + arg(act) + ", " + arg(pre) + ", " + arg(post) +
                            ", " + slotExpr(idx) + ");";
                else
                    stmt += " = gala::gcn_aggregate_apply(" + X + ", " + arg(pre) + ", " + arg(post) + ", " + slotExpr(idx) + ");";
                replaceSpans(fwd, sp, j, last, stmt);
                done = last + 1;
                k = last;
                break;
            }
        }
    }

    // The base emits a GAT layer (common.h:622-894, 1175-1184) as four steps over E-long
    // edge tensors: the edge sum's autograd class (K5), torch's LeakyReLU, the softmax class
    // (torch exp / clamp / reciprocal around K7 and K8) and the attention-weighted aggregation
    // class -- with their backwards (K9, the softmax backward's torch ops around K7 / K8, K7 for
    // the logits' gradient): on the Products shape 30.8 ms per epoch where galac's fused layer
    // takes 20.8 (profiles/r05_refgen_gat_products.jsonl).  The node chain
    //     AGGREGATE_EDGE_SUM(L, R, graph) -> LEAKY_RELU -> SOFTMAX -> AGGREGATE_MUL_SUM(X, attn)
    // (the aggregation in the base's attention form, every node on slot 0, `attn` read by
    // nothing after the chain) becomes the mirror's fused layer over the same slot in REF mode,
    //     res = gala::gat_aggregate_apply(L, R, X, li, 0.2, GALA_SOFTMAX_REF);
    // (the same chain of operations per edge, one pass per row; alpha = p * q with the
    // reference's clamp, 1e-12 and sequential row sums; gradients d aL = d aR = the row sums of
    // the LeakyReLU'd softmax gradient, as the base's classes return them; the slope is the
    // base's LeakyReLU module's, 0.2 whatever the node's parameter, common.h:1180).  When R is
    // the FFN_OP_EDGE of the aggregated rows X themselves (efcN, emitted as the head-attention
    // op), the layer recomputes it from the rows it gathers (gat_aggregate_ffn_apply, galac's
    // spelling) and R's statement goes when nothing else reads R.  The values are the chain's
    // within fp32 rounding, not bit for bit: the fused kernels sum in the chain's order but
    // round alpha = p * q once per edge where the chain stores it (tests/test_gpu_refgen.py
    // checks the program against galac's IR in float64 at 1e-4 and against the base's spelling,
    // GALA_REFGEN_UNFUSED).
    void fuseGatChains(Code &fwd, const std::vector<Span> &sp) {
        for (size_t k = 3; k < sp.size(); ++k) {
            const Span &ag = sp[k], &sm = sp[k - 1], &lr = sp[k - 2], &es = sp[k - 3];
            if (opOf(ag) != AGGREGATE_MUL_SUM_OP || !ag.edgeUpdate || sampled(ag.node) || ag.last == ag.first) continue;
            if (opOf(sm) != NON_LNR_OP_SOFTMAX || out(sm) != "attn") continue;   // the aggregation reads `attn`
            if (opOf(lr) != NON_LNR_OP_LEAKY_RELU || out(lr) != in(sm, 0)) continue;
            if (opOf(es) != AGGREGATE_EDGE_SUM_OP || out(es) != in(lr, 0)) continue;
            if (ag.node->getInput(1)->getDataInfo()->getIndex() != 0 || es.node->getInput(2)->getDataInfo()->getIndex() != 0)
                continue;   // a subgraph slot off validation epochs: the base's spelling
            bool dead = !readLater(fwd, sp, k, "attn");
            for (const std::string &v : {out(es), out(lr)})
                dead = dead && (v == "attn" || !readLater(fwd, sp, k, v));
            if (!dead) continue;
            const std::string X = in(ag, 0), L = in(es, 0), R = in(es, 1);
            // R = efcN(X) just before, with only other attention Linears (not assigning X) between
            long h = -1;
            for (long i = (long)k - 4; i >= 0; --i) {
                if (opOf(sp[i]) != FFN_OP_EDGE || out(sp[i]) == X) break;
                if (out(sp[i]) == R) {
                    if (in(sp[i], 0) == X) h = i;
                    break;
                }
            }
            const std::string res = out(ag), head = "\n        // EDGE SUM / LEAKY RELU / SOFTMAX / AGGREGATE fused (HIPGenerator)\n        ";
            std::string call;
            if (h >= 0 && R != L) {
                const std::string W = "efc" + std::to_string(sp[h].fcEdge);
                call = res + " = gala::gat_aggregate_ffn_apply(" + L + ", " + X + ", " + W + "->weight, " + W +
                       "->bias, 0, 0.2, GALA_SOFTMAX_REF);";
                if (!readLater(fwd, sp, k, R))
                    for (int e = sp[h].first; e < sp[h].last; ++e) fwd.atLine(e)->clear();
            } else {
                call = res + " = gala::gat_aggregate_apply(" + L + ", " + R + ", " + X + ", 0, 0.2, GALA_SOFTMAX_REF);";
            }
            // the LeakyReLU module's declaration (the span's first entry when it has two) stays:
            // later layers' calls use the variable
            const std::string decl = lr.last - lr.first == 2 ? *fwd.atLine(lr.first) : std::string();
            replaceSpans(fwd, sp, k - 3, k, head + call);
            if (!decl.empty()) *fwd.atLine(lr.first) = decl;
        }
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

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

    void dataPrep(std::vector<CIRNode *> &program) override {
        std::string s =
            "  torch::Device device = gala_program_device();\n"
            "  auto options_cu_int = torch::TensorOptions().dtype(torch::kInt).requires_grad(false).device(device);\n"
            "  auto options_cu_float_grad = torch::TensorOptions().dtype(torch::kFloat).requires_grad(true).device(device);\n"
            "  auto options_cu_float_ngrad = torch::TensorOptions().dtype(torch::kFloat).requires_grad(false).device(device);\n"
            "  auto options_cu_bool = torch::TensorOptions().dtype(torch::kBool).requires_grad(false).device(device);\n"
            "  auto options_cu_long = torch::TensorOptions().dtype(torch::kLong).device(device);\n"
            "  // features, labels and masks: host matrices copied into torch-owned device tensors\n"
            "  torch::Tensor t_iden = torch::from_blob(input_emb.vals_ptr(), {(int64_t)nrows, (int64_t)emb_size},\n"
            "                                         torch::kFloat).to(device).clone().requires_grad_(true);\n"
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
    // The attention Linears (efcN, one output per head) stay as they are.
    static void denseOnMatrixCores(Code &code) {
        for (int i = 0; i < code.getNum(); ++i) {
            std::string *l = code.atLine(i);
            for (const std::string pre : {"sfc", "fc"}) {
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
                    l->replace(p, e + 1 - p, "gala::ffn_apply(" + arg + ", " + mod + "->weight, " + mod + "->bias)");
                }
            }
        }
    }

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

// Python module `apex_example_amd._C`.
//
// Submodules mirror the Apex extension names so the Python layer can expose
// drop-in facades: amp_C (multi-tensor ops), apex_C (flatten/unflatten),
// fused_layer_norm_cuda, syncbn, plus `reducer` (the DDP core).
#include <torch/extension.h>

#include "amd_kernels.h"
#include "amp_ops.h"
#include "attn_ops.h"
#include "norm_ops.h"
#include "pool_ops.h"
#include "dense_ops.h"
#include "lt_ops.h"
#include "xent_ops.h"
#include "emb_ops.h"
#include "reducer.h"

#include <hip/hip_runtime_api.h>

#include <cstdint>
#include <vector>

namespace py = pybind11;
using namespace amd;

static at::Tensor flatten_dense(const std::vector<at::Tensor>& ts) {
  std::vector<at::Tensor> flat;
  flat.reserve(ts.size());
  for (auto& t : ts) flat.push_back(t.contiguous().view({-1}));
  if (flat.empty()) return at::empty({0});
  return at::cat(flat);
}

static std::vector<at::Tensor> unflatten_dense(const at::Tensor& flat,
                                               const std::vector<at::Tensor>& like) {
  std::vector<at::Tensor> out;
  out.reserve(like.size());
  int64_t off = 0;
  for (auto& t : like) {
    int64_t n = t.numel();
    out.push_back(flat.narrow(0, off, n).view(t.sizes()));
    off += n;
  }
  return out;
}

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "MI355X-native kernels for apex_example_amd (gfx950)";
  m.attr("arch") = "gfx950";

  auto mt = m.def_submodule("mt", "multi-tensor apply ops (device-resident launch tables)");
  mt.def("scale", &mt_scale_op, py::arg("noop"), py::arg("lists"), py::arg("scale"),
         py::arg("scale_t") = py::none(), py::arg("invert") = false);
  mt.def("scale_any", &mt_scale_any_op, py::arg("noop"), py::arg("lists"), py::arg("scale"),
         py::arg("scale_t") = py::none(), py::arg("invert") = false);
  mt.def("check_finite", &mt_check_finite_op);
  mt.def("axpby", &mt_axpby_op);
  mt.def("zero", &mt_zero_op);
  mt.def("copy_if", &mt_copy_if_op);
  mt.def("norm", &mt_norm_op, py::arg("noop"), py::arg("list"), py::arg("per_tensor") = false,
         py::arg("max_norm") = false);
  mt.def("sgd", &mt_sgd_op);
  mt.def("adam", &mt_adam_op);
  mt.def("lamb", &mt_lamb_op);
  mt.def("lamb_legacy_stage1", &mt_lamb_legacy_stage1_op);
  mt.def("lamb_legacy_stage2", &mt_lamb_legacy_stage2_op);
  mt.def("novograd", &mt_novograd_op);
  mt.def("adagrad", &mt_adagrad_op);
  mt.def("update_loss_scale", &update_loss_scale_op, py::arg("scale"), py::arg("unskipped"),
         py::arg("skipped"), py::arg("overflow"), py::arg("factor"), py::arg("window"),
         py::arg("min_scale"), py::arg("max_scale"), py::arg("dynamic"),
         py::arg("applied") = py::none());
  mt.def("advance_step", &advance_step_op);
  mt.def("mark_step_done", &mark_step_done_op);
  mt.def("flat_scale", &flat_scale_op);
  py::class_<StepPlan, std::shared_ptr<StepPlan>>(mt, "StepPlan")
      .def(py::init<std::vector<at::Tensor>, TensorLists>(), py::arg("owners"), py::arg("fixed"))
      .def("refresh", &StepPlan::refresh)
      .def("set_absent", &StepPlan::set_absent)
      .def("sgd", &StepPlan::sgd)
      .def("sgd_pair", &StepPlan::sgd_pair)
      .def("adam", &StepPlan::adam)
      .def("grad_norm_into", &StepPlan::grad_norm_into)
      .def("lamb", &StepPlan::lamb)
      .def("size", &StepPlan::size)
      .def("rebuilds", &StepPlan::rebuilds);
  mt.def("plan_cache_clear", &mt_plan_cache_clear);
  mt.def("plan_cache_size", &mt_plan_cache_size);

  auto ac = m.def_submodule("apex_C", "flatten / unflatten (apex_C parity)");
  ac.def("flatten", &flatten_dense);
  ac.def("unflatten", &unflatten_dense);

  auto ln = m.def_submodule("layer_norm", "fused LayerNorm / RMSNorm (wave64 row kernels)");
  ln.def("forward", &layer_norm_forward_op);
  ln.def("backward", &layer_norm_backward_op);
  ln.def("add_dropout_forward", &add_dropout_layer_norm_forward_op);
  ln.def("add_dropout_backward", &add_dropout_layer_norm_backward_op);
  ln.def("set_bwd_one_row", &layer_norm_bwd_one_row);
  ln.def("bwd_one_row", &layer_norm_bwd_one_row_on);

  auto attn = m.def_submodule("attn", "fused attention (head dim 64, MFMA, gfx950)");
  attn.def("fwd", &attn_fwd_op);
  attn.def("bwd", &attn_bwd_op);

  auto dn = m.def_submodule("dense", "dense-layer bias gradients / fused GELU backward");
  dn.def("bias_grad", &bias_grad_op);
  dn.def("gelu_bwd_bias_grad", &gelu_bwd_bias_grad_op);
  dn.def("act_bwd_bias_grad", &act_bwd_bias_grad_op);
  dn.def("gelu", &gelu_fwd_op);
  dn.def("gelu_fwd_lt", &dense_gelu_fwd_op);
  dn.def("dgelu_bgrad_lt", &dense_dgelu_bgrad_op);
  dn.def("lt_cache_clear", &lt_algo_cache_clear);
  dn.def("lt_probe", &lt_probe_op);
  dn.def("wgrad_bgrad_lt", &dense_wgrad_bgrad_op);
  dn.def("gemm4w", &gemm4w_op, py::arg("a"), py::arg("b"), py::arg("epi") = 0,
         py::arg("bias") = py::none(), py::arg("aux") = py::none(), py::arg("want_pre") = false,
         py::arg("tanh") = false, py::arg("bias_grad_dtype") = py::none());
  dn.def("gemm4w_ok", &gemm4w_ok);
  dn.def("wgrad4w", &wgrad4w_op, py::arg("dy"), py::arg("x"), py::arg("splits"),
         py::arg("out_dtype"), py::arg("out") = py::none(), py::arg("accumulate") = true);
  dn.def("wgrad4w_ok", &wgrad4w_ok);
  dn.def("wgrad4w_bias", &wgrad4w_bias_op, py::arg("dy"), py::arg("x"), py::arg("splits"),
         py::arg("out_dtype"), py::arg("out") = py::none(), py::arg("accumulate") = true,
         py::arg("bias_dtype") = at::kFloat);
  auto xe = m.def_submodule("xentropy", "fused softmax cross entropy + label smoothing");
  xe.def("forward", &xentropy_fwd_op);
  xe.def("backward", &xentropy_bwd_op);

  auto emb = m.def_submodule("emb", "deterministic embedding weight gradient (no host sync)");
  emb.def("wgrad", &embedding_wgrad_op, py::arg("idx"), py::arg("dy"), py::arg("V"),
          py::arg("padding_idx"), py::arg("out_dtype"));

  auto pool = m.def_submodule("pool", "NHWC max pooling (gather backward, no atomics)");
  pool.def("max_fwd", &maxpool2d_nhwc_fwd_op);
  pool.def("max_bwd", &maxpool2d_nhwc_bwd_op);
  pool.def("max_bwd_bn", &maxpool2d_nhwc_bwd_bn_op, py::arg("dy"), py::arg("idx"), py::arg("H"),
           py::arg("W"), py::arg("x"), py::arg("mean"), py::arg("invstd"),
           py::arg("weight") = py::none(), py::arg("bias") = py::none());
  pool.def("gap_bwd", &gap_nhwc_bwd_op, py::arg("dy"), py::arg("H"), py::arg("W"));
  pool.def("max_fwd_bn", &maxpool2d_nhwc_bn_fwd_op);
  auto conv = m.def_submodule("conv", "MFMA implicit-GEMM convolutions (NHWC bf16)");
  conv.def("conv_fwd", &conv_nhwc_fwd_op, py::arg("x"), py::arg("w"), py::arg("stride") = 1);
  conv.def("conv_fwd_bnbwd", &conv_nhwc_fwd_bnbwd_op, py::arg("dy"), py::arg("w"),
           py::arg("add"), py::arg("x"), py::arg("rmask"), py::arg("mean"), py::arg("invstd"),
           py::arg("bn_weight"), py::arg("bn_bias"), py::arg("relu_mode"),
           py::arg("add_stride2") = false);
  conv.def("conv_fwd_stats", &conv_nhwc_fwd_stats_op, py::arg("x"), py::arg("w"),
           py::arg("stride") = 1, py::arg("shift") = py::none());
  conv.def("conv_dgrad_s2", &conv_nhwc_dgrad_s2_op);
  conv.def("conv_dgrad_s2_bnbwd", &conv_nhwc_dgrad_s2_bnbwd_op, py::arg("dy"), py::arg("wt"),
           py::arg("H"), py::arg("W"), py::arg("x"), py::arg("rmask"), py::arg("mean"),
           py::arg("invstd"), py::arg("bn_weight"), py::arg("bn_bias"), py::arg("relu_mode"));
  conv.def("conv_wgrad", &conv_nhwc_wgrad_op, py::arg("dy"), py::arg("x"), py::arg("out_dtype"),
           py::arg("algo") = 0, py::arg("stride") = 1, py::arg("ksize") = 3,
           py::arg("out") = py::none(), py::arg("accumulate") = true);
  conv.def("splitk_reduce", &splitk_reduce_op, py::arg("part"), py::arg("out_dtype"),
           py::arg("out") = py::none(), py::arg("accumulate") = true);
  conv.def("stem_pad", &stem_pad_op);
  conv.def("stem_fwd", &stem_fwd_op);
  conv.def("stem_fwd_stats", &stem_fwd_stats_op, py::arg("xp"), py::arg("wk"),
           py::arg("shift") = py::none());
  conv.def("stem_wgrad", &stem_wgrad_op);
  conv.def("rot_weight", &conv3x3_rot_weight_op);
  conv.def("transpose_weight", &conv1x1_transpose_weight_op);
  conv.def("prep_weights", &conv_prep_weights_op);
  conv.def("set_nfast", &conv_nfast, py::arg("mode"));
  conv.def("set_halo_nfast", &conv_halo_nfast, py::arg("on"));
  conv.def("set_halo", &conv_halo_enable, py::arg("mode"),
           "3x3 stride-1 convs on the halo-resident kernel: 0 off, 1 auto, 64 / 128 force "
           "that output-tile width where possible");
  conv.def("halo_enabled", &conv_halo_enabled);
  conv.def("set_halo_mtile", &conv_halo_mtile, py::arg("bm"));
  conv.def("set_bnbwd_early", &conv_bnbwd_early);
  conv.def("set_1x1_gemm4w", &conv_1x1_gemm4w);
  conv.def("on_gemm4w_1x1", &conv_1x1_on_gemm4w, py::arg("M"), py::arg("Cin"), py::arg("Cout"));

  auto bn = m.def_submodule("bn", "BatchNorm / SyncBatchNorm kernels (NCHW + NHWC)");
  bn.def("local_stats", &bn_local_stats_op);
  bn.def("train_stats", &bn_train_stats_op);
  bn.def("combine_stats", &bn_combine_stats_op);
  bn.def("apply", &bn_apply_op);
  bn.def("forward_local", &bn_forward_local_op, py::arg("x"), py::arg("weight"),
         py::arg("bias"), py::arg("running_mean"), py::arg("running_var"), py::arg("nbt"),
         py::arg("eps"), py::arg("momentum"), py::arg("z"), py::arg("relu"),
         py::arg("want_mask") = false);
  bn.def("apply_mask", &bn_apply_mask_op);
  bn.def("slab_train_stats", &bn_slab_train_stats_op, py::arg("slab"), py::arg("count"),
         py::arg("shift"), py::arg("running_mean"), py::arg("running_var"), py::arg("nbt"),
         py::arg("eps"), py::arg("momentum"));
  bn.def("slab_reduce_grad", &bn_slab_reduce_grad_op, py::arg("slab"), py::arg("invstd"),
         py::arg("weight"), py::arg("need_wgrad"), py::arg("sum_scale") = py::none(),
         py::arg("grad_weight") = py::none(), py::arg("grad_bias") = py::none(),
         py::arg("accumulate") = true);
  bn.def("slab_packed_stats", &bn_slab_packed_stats_op, py::arg("slab"), py::arg("count"),
         py::arg("shift"), py::arg("out") = py::none());
  bn.def("set_tuning", &bn_set_tuning, py::arg("red_rpt") = -1, py::arg("red_cap") = -1,
         py::arg("red_min") = -1, py::arg("elem_rpt") = -1, py::arg("elem_cap") = -1,
         py::arg("elem_min") = -1);
  bn.def("get_tuning", []() {
    int o[6];
    bn_get_tuning(o);
    return std::vector<int>(o, o + 6);
  });
  bn.def("reduce_grad", &bn_reduce_grad_op, py::arg("dy"), py::arg("x"), py::arg("mean"),
         py::arg("invstd"), py::arg("weight"), py::arg("bias"), py::arg("z"), py::arg("relu"),
         py::arg("need_wgrad"), py::arg("mask") = py::none(),
         py::arg("sum_scale") = py::none(), py::arg("grad_weight") = py::none(),
         py::arg("grad_bias") = py::none(), py::arg("accumulate") = true);
  bn.def("local_stats_packed", &bn_local_stats_packed_op, py::arg("x"),
         py::arg("out") = py::none());
  bn.def("combine_stats_sync", &bn_combine_stats_sync_op, py::arg("gathered"), py::arg("eps"),
         py::arg("momentum"), py::arg("running_mean"), py::arg("running_var"),
         py::arg("nbt") = py::none());
  bn.def("backward_elemt", &bn_backward_elemt_op, py::arg("dy"), py::arg("x"), py::arg("mean"),
         py::arg("invstd"), py::arg("weight"), py::arg("bias"), py::arg("sum_dy"),
         py::arg("sum_dy_xmu"), py::arg("count"), py::arg("z"), py::arg("relu"),
         py::arg("want_dz"), py::arg("mask") = py::none());

  bn.def("backward_x2_ok", &bn_backward_x2_ok);
  bn.def("apply2_mask", &bn_apply2_mask_op, py::arg("x"), py::arg("mean"), py::arg("invstd"),
         py::arg("weight"), py::arg("bias"), py::arg("xz"), py::arg("meanz"), py::arg("invstdz"),
         py::arg("weightz"), py::arg("biasz"));
  bn.def("backward_elemt_x2", &bn_backward_elemt_x2_op, py::arg("dy"), py::arg("x"),
         py::arg("mean"), py::arg("invstd"), py::arg("weight"), py::arg("bias"),
         py::arg("sum_dy"), py::arg("sum_dy_xmu"), py::arg("count"), py::arg("x2"),
         py::arg("mean2"), py::arg("invstd2"), py::arg("weight2"), py::arg("need_wgrad2"));
  bn.def("backward_local", &bn_backward_local_op, py::arg("dy"), py::arg("x"), py::arg("mean"),
         py::arg("invstd"), py::arg("weight"), py::arg("bias"), py::arg("z"), py::arg("relu"),
         py::arg("need_wgrad"), py::arg("want_dz"), py::arg("mask") = py::none());

  auto rd = m.def_submodule("reducer", "DDP bucketed gradient reducer core");
  register_reducer(rd);
}

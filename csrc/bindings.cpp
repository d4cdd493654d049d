// Python bindings for the distlearn MI355X native library (pybind11).
// Module: torch_distlearn_amd._C
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "comm/communicator.h"
#include "dl_ops.h"
#include "runtime/loader.h"

namespace py = pybind11;
using namespace dl;

PYBIND11_MODULE(_C, m) {
  m.doc() = "distlearn MI355X (gfx950) native kernels, RCCL communicator and data runtime";

  // ---- flat bucket kernels --------------------------------------------------
  m.def("sgd_update", &sgd_update, py::arg("p"), py::arg("g"), py::arg("mom"), py::arg("p16"), py::arg("slot"),
        py::arg("lr"), py::arg("momentum"), py::arg("wd"), py::arg("n"), py::arg("stream"));
  m.def("scale_by_count", &scale_by_count);
  m.def("elastic_step", &elastic_step);
  m.def("elastic_step_wire16", &elastic_step_wire16);
  m.def("add_inplace", &add_inplace);
  m.def("fill_f32", &fill_f32);
  m.def("cast_f32_bf16", &cast_f32_bf16);
  m.def("stamp_time", &stamp_time);
  m.def("wall_clock_khz", &wall_clock_khz);
  m.def("cast_bf16_f32", &cast_bf16_f32);
  m.def("sgd_update_g16", &sgd_update_g16);
  m.def("sgd_update_slabs", &sgd_update_slabs);
  m.def("arm_sgd_next_prep", &arm_sgd_next_prep);
  m.def("sgd_next_prep_armed", &sgd_next_prep_armed);
  m.def("set_sgd_trim", &set_sgd_trim);
  m.def("disarm_sgd_next_prep", &disarm_sgd_next_prep);
  m.def("set_conv_side_sgd", &set_conv_side_sgd);
  m.def("set_conv_side_reduce", &set_conv_side_reduce);
  m.def("slab_reduce_multi", &slab_reduce_multi);
  m.def("confusion_update", &confusion_update);
  m.def("bn_nhwc_fwd", &bn_nhwc_fwd);
  m.def("bn_nhwc_bwd", &bn_nhwc_bwd);
  m.def("set_bn_reduce_blocks", &set_bn_reduce_blocks);
  m.def("set_bn_tuning", &set_bn_tuning);
  m.def("set_bn_minw", &set_bn_minw);
  m.def("bn_rows_reduce", &bn_rows_reduce);
  m.def("bn_nhwc_fwd_pad", &bn_nhwc_fwd_pad, py::arg("x"), py::arg("res"), py::arg("y"), py::arg("acc"), py::arg("w"),
        py::arg("b"), py::arg("save"), py::arg("run_mean"), py::arg("run_var"), py::arg("M"), py::arg("C"),
        py::arg("eps"), py::arg("momentum"), py::arg("relu"), py::arg("have_stats"), py::arg("H"), py::arg("W"),
        py::arg("opad"), py::arg("stream"), py::arg("mbits") = 0, py::arg("rbn_acc") = 0, py::arg("rbn_w") = 0,
        py::arg("rbn_b") = 0, py::arg("rbn_save") = 0, py::arg("rbn_rm") = 0, py::arg("rbn_rv") = 0,
        py::arg("rbn_eps") = 1e-5, py::arg("rbn_momentum") = 0.1);
  m.def("bn_nhwc_bwd_pad", &bn_nhwc_bwd_pad, py::arg("dy"), py::arg("y"), py::arg("x"), py::arg("save"),
        py::arg("w"), py::arg("b"), py::arg("acc"), py::arg("dx"), py::arg("dres"), py::arg("dw"), py::arg("db"),
        py::arg("M"), py::arg("C"), py::arg("relu"), py::arg("H"), py::arg("W"), py::arg("opad"), py::arg("stream"),
        py::arg("have_sums") = 0, py::arg("mbits") = 0, py::arg("rbn_x") = 0, py::arg("rbn_save") = 0,
        py::arg("rbn_w") = 0, py::arg("rbn_acc") = 0, py::arg("rbn_dw") = 0, py::arg("rbn_db") = 0);
  m.def("zero_border_nhwc", &zero_border_nhwc);
  m.def("gather_normalize", &gather_normalize);

  // ---- convnet kernels (MFMA implicit GEMM, BN/ReLU/pool, classifier head) ------
  m.def("conv_fwd", &conv_fwd);
  m.def("conv_fwd_add", &conv_fwd_add, py::arg("x"), py::arg("w"), py::arg("y"), py::arg("addend"), py::arg("B"),
        py::arg("H"), py::arg("W"), py::arg("Cin"), py::arg("Cout"), py::arg("KS"), py::arg("tile"), py::arg("stream"),
        py::arg("addend_mask") = 0);
  m.def("conv_fwd_stat_rows", &conv_fwd_stat_rows);
  m.def("set_conv_region", &set_conv_region);
  m.def("set_conv_region_stages", &set_conv_region_stages);
  m.def("set_bn_bwd_items", &set_bn_bwd_items);
  m.def("set_conv_region_ablate", &set_conv_region_ablate);
  m.def("set_conv_region_waves", &set_conv_region_waves);
  m.def("set_conv_stages", &set_conv_stages);
  m.def("set_conv_posm", &set_conv_posm);
  m.def("set_conv_c8_mt", &set_conv_c8_mt);
  m.def("set_conv_waves", &set_conv_waves);
  m.def("set_conv_debug", &set_conv_debug);
  m.def("conv_wgrad", &conv_wgrad);
  m.def("combine_bwd_reduce", &combine_bwd_reduce);
  m.def("bn_bwd_apply_head", &bn_bwd_apply_head);
  m.def("combine_bwd_reduce_blocks", &combine_bwd_reduce_blocks);
  m.def("conv_fwd_ex", &conv_fwd_ex);
  m.def("conv_fwd_bnred", &conv_fwd_bnred);
  m.def("conv_fwd_fix", &conv_fwd_fix);
  m.def("conv_fix_ok", &conv_fix_ok);
  m.def("conv_region_ok", &conv_region_ok, py::arg("B"), py::arg("H"), py::arg("W"), py::arg("Cin"), py::arg("Cout"),
        py::arg("KS"), py::arg("tile"), py::arg("splits") = 1);
  m.def("set_conv_fwd_pf", &set_conv_fwd_pf);
  m.def("set_head_stamps", &set_head_stamps);
  m.def("set_bn_stamps", &set_bn_stamps);
  m.def("set_conv_wgrad_stamps", &set_conv_wgrad_stamps);
  m.def("conv_wgrad_ex", &conv_wgrad_ex);
  // ---- ResNet-50 glue (resnet_glue.hip) ------------------------------------------
  m.def("s2d_stem_input", &s2d_stem_input);
  m.def("stem_weight_pack", &stem_weight_pack);
  m.def("stem_wgrad_unpack", &stem_wgrad_unpack);
  m.def("phase_weights", &phase_weights);
  m.def("head_pool", &head_pool);
  m.def("head_softmax_nll", &head_softmax_nll);
  m.def("head_weight_prep", &head_weight_prep);
  m.def("head_broadcast", &head_broadcast);
  m.def("head_wgrad_reduce", &head_wgrad_reduce);
  m.def("slab_reduce", &slab_reduce);
  m.def("slab_reduce_add", &slab_reduce_add);
  m.def("slab_reduce_add_oihw", &slab_reduce_add_oihw);
  m.def("weight_flip_transpose", &weight_flip_transpose);
  m.def("transpose_many", &transpose_many);
  m.def("transpose_entry_bytes", &transpose_entry_bytes);
  m.def("weights_to_cl", &weights_to_cl);
  m.def("cl_entry_bytes", &cl_entry_bytes);
  m.def("pack_weight", &pack_weight);
  m.def("pad_channels", &pad_channels);
  m.def("prep_step", &prep_step);
  m.def("prep_step_gather", &prep_step_gather);
  m.def("bn_finalize", &bn_finalize);
  m.def("bn_relu_pool_fwd", &bn_relu_pool_fwd);
  m.def("bn_bwd_blocks", &bn_bwd_blocks);
  m.def("bn_relu_pool_bwd_reduce", &bn_relu_pool_bwd_reduce);
  m.def("bn_bwd_finalize", &bn_bwd_finalize);
  m.def("bn_relu_pool_bwd_apply", &bn_relu_pool_bwd_apply);
  m.def("bn_relu_pool_bwd_apply_sums", &bn_relu_pool_bwd_apply_sums);
  m.def("bn_relu_pool_fwd_fin", &bn_relu_pool_fwd_fin);
  // reduction mode of the BN statistics / gradients: 0 = deterministic partial
  // rows + finalize kernels; R >= 1 (power of two) = atomic per-channel totals
  // striped over R rows, no finalize launches.  reduce_atomic() returns R.
  m.def("set_reduce_atomic", [](int rows) {
    set_reduce_atomic_conv(rows);
    set_reduce_atomic_bn(rows);
  });
  m.def("reduce_atomic", []() { return reduce_rows(); });
  m.def("set_bn_fin_grid", &set_bn_fin_grid);
  m.def("head_fwd_bwd", &head_fwd_bwd);
  m.def("head_fwd_bwd_pool", &head_fwd_bwd_pool);
  m.def("head_fwd_bwd_pool_wt", &head_fwd_bwd_pool_wt);
  m.def("bn_bwd_reduce_head", &bn_bwd_reduce_head);
  m.def("bn_bwd_reduce_slab", &bn_bwd_reduce_slab);
  m.def("head_wgrad", &head_wgrad);
  m.def("mnist_step", &mnist_step);
  m.def("mnist_scratch_bytes", &mnist_scratch_bytes);
  m.def("maxpool_bn_bwd", &maxpool_bn_bwd);
  m.def("maxpool_nhwc_fwd", &maxpool_nhwc_fwd, py::arg("x"), py::arg("y"), py::arg("idx"), py::arg("N"), py::arg("H"),
        py::arg("W"), py::arg("C"), py::arg("K"), py::arg("S"), py::arg("P"), py::arg("stream"), py::arg("bn_acc") = 0,
        py::arg("bn_w") = 0, py::arg("bn_b") = 0, py::arg("bn_save") = 0, py::arg("bn_rm") = 0, py::arg("bn_rv") = 0,
        py::arg("bn_eps") = 1e-5, py::arg("bn_momentum") = 0.1);
  m.def("maxpool_nhwc_bwd", &maxpool_nhwc_bwd);

  // ---- RCCL communicator ------------------------------------------------------
  m.def("rccl_unique_id", []() { return py::bytes(rccl_unique_id()); });
  m.def("rccl_version", &rccl_version);
  py::class_<RcclCommunicator>(m, "RcclCommunicator")
      .def(py::init([](py::bytes uid, int rank, int world, int device, double timeout_s, int max_ctas) {
             std::string id(uid);  // copy while holding the GIL
             py::gil_scoped_release nogil;  // ncclCommInitRank blocks on the other ranks
             return new RcclCommunicator(id, rank, world, device, timeout_s, max_ctas);
           }),
           py::arg("uid"), py::arg("rank"), py::arg("world"), py::arg("device"), py::arg("timeout_s") = 0.0,
           py::arg("max_ctas") = 0)
      .def_property_readonly("max_ctas", &RcclCommunicator::max_ctas)
      .def_property_readonly("rank", &RcclCommunicator::rank)
      .def_property_readonly("world", &RcclCommunicator::world)
      .def_property_readonly("device", &RcclCommunicator::device)
      .def("all_reduce", &RcclCommunicator::all_reduce)
      .def("broadcast", &RcclCommunicator::broadcast)
      .def("reduce", &RcclCommunicator::reduce)
      .def("reduce_scatter", &RcclCommunicator::reduce_scatter)
      .def("all_gather", &RcclCommunicator::all_gather)
      .def("send", &RcclCommunicator::send)
      .def("recv", &RcclCommunicator::recv)
      .def("group_start", &RcclCommunicator::group_start)
      .def("group_end", &RcclCommunicator::group_end)
      .def("track", &RcclCommunicator::track)
      .def("set_paused", &RcclCommunicator::set_paused, py::call_guard<py::gil_scoped_release>())
      .def("polls", &RcclCommunicator::polls)
      .def("set_timeout", &RcclCommunicator::set_timeout)
      .def("timeout", &RcclCommunicator::timeout)
      .def("pending", &RcclCommunicator::pending)
      .def("inflight", &RcclCommunicator::inflight)
      .def("error", &RcclCommunicator::error)
      .def("async_error", &RcclCommunicator::async_error)
      .def("destroy", &RcclCommunicator::destroy, py::call_guard<py::gil_scoped_release>())
      .def("abort", &RcclCommunicator::abort, py::call_guard<py::gil_scoped_release>());

  // ---- data runtime -------------------------------------------------------------
  py::class_<PartitionSampler>(m, "PartitionSampler")
      .def(py::init<int64_t, std::vector<int64_t>, int, int, int, int, uint64_t>(), py::arg("n"), py::arg("labels"),
           py::arg("num_classes"), py::arg("partition"), py::arg("partitions"), py::arg("kind"), py::arg("seed"))
      .def("size", &PartitionSampler::size)
      .def("num_batches", &PartitionSampler::num_batches)
      .def("reset_epoch", &PartitionSampler::reset_epoch)
      .def("next_batch", [](PartitionSampler& s, uintptr_t out, int64_t batch) {
        return s.next_batch(reinterpret_cast<int64_t*>(out), batch);
      });
}

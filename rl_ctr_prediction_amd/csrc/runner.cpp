// The per-step launch sequence of a single-process training step, issued in one call.
//
// The reference trains one batch per loop iteration (all_main/pretrain_main.py:71-78:
// forward, BCELoss, backward, optimizer.step). Here that iteration is a captured HIP graph
// per input slot (rl_ctr_prediction_amd/trainer.py InputSlot), and what remains on the host
// per batch is a fixed sequence of runtime calls: wait for the slot's staged ids, copy the
// labels in, launch the step graph, and stage the next batch(es) — copy their ids into
// their slots and launch their sparse-plan graphs on the plan streams. Issued from Python
// as separate torch calls that sequence cost ~60 us of host time per step, more than the
// GPU needs for a C2 step (FM, 4096 x 26); one ctypes call here costs a few us.
//
// Host code only (HIP runtime calls; no kernels, no allocation, no synchronisation).
#include "ctr_common.h"

extern "C" int ctr_step_launch(ctr_stream_t main_stream, void* wait_event, const void* y_src,
                               void* y_dst, int64_t y_bytes, void* step_graph,
                               void* start_event, const ctr_stage* stages, int n_stages) {
  CTR_REQUIRE(step_graph && n_stages >= 0 && (n_stages == 0 || (stages && start_event)) &&
                  y_bytes >= 0 && (y_bytes == 0 || (y_src && y_dst)),
              "ctr_step_launch: bad arguments");
  for (int i = 0; i < n_stages; ++i)
    CTR_REQUIRE(stages[i].stream && stages[i].done_event && stages[i].bytes >= 0 &&
                    (stages[i].bytes == 0 || (stages[i].src && stages[i].dst)),
                "ctr_step_launch: bad stage %d", i);
  hipStream_t m = ctr::as_stream(main_stream);
  // everything enqueued on the main stream before this step: the last readers of the
  // slots the stages overwrite
  if (n_stages > 0) CTR_HIP_CHECK(hipEventRecord(static_cast<hipEvent_t>(start_event), m));
  if (wait_event) CTR_HIP_CHECK(hipStreamWaitEvent(m, static_cast<hipEvent_t>(wait_event), 0));
  if (y_bytes > 0)
    CTR_HIP_CHECK(hipMemcpyAsync(y_dst, y_src, (size_t)y_bytes, hipMemcpyDeviceToDevice, m));
  CTR_HIP_CHECK(hipGraphLaunch(static_cast<hipGraphExec_t>(step_graph), m));
  // the stages after the step graph (issued before it, the next batch's plan overlapped the
  // step's first kernels and measured slower: C2 44.4 / 48.5 vs 49.1 / 52.2 M ex/s)
  for (int i = 0; i < n_stages; ++i) {
    const ctr_stage& s = stages[i];
    hipStream_t ps = ctr::as_stream(s.stream);
    CTR_HIP_CHECK(hipStreamWaitEvent(ps, static_cast<hipEvent_t>(start_event), 0));
    if (s.bytes > 0)
      CTR_HIP_CHECK(hipMemcpyAsync(s.dst, s.src, (size_t)s.bytes, hipMemcpyDeviceToDevice, ps));
    if (s.plan_graph) CTR_HIP_CHECK(hipGraphLaunch(static_cast<hipGraphExec_t>(s.plan_graph), ps));
    CTR_HIP_CHECK(hipEventRecord(static_cast<hipEvent_t>(s.done_event), ps));
  }
  return CTR_OK;
}

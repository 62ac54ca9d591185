// Captured launches (hipGraph) for StepGraph (powergridworld_amd/graph.py):
// the library's launches issued on a stream between pgw_graph_begin and
// pgw_graph_end become one executable graph, launched per call with
// pgw_graph_launch -- one runtime call per replay, from the caller's thread,
// without the bookkeeping a framework's graph object adds around it.
#include "pgw_common.h"

using namespace pgw;

extern "C" {

int32_t pgw_graph_begin(void* stream) {
  PGW_REQUIRE(stream, "pgw_graph_begin: capture needs a created stream, not the null stream");
  if (hipStreamBeginCapture(static_cast<hipStream_t>(stream), hipStreamCaptureModeThreadLocal) != hipSuccess) {
    set_error("pgw_graph_begin: hipStreamBeginCapture failed");
    return PGW_ERR_HIP;
  }
  return PGW_OK;
}

int32_t pgw_graph_end(void* stream, void** exec_out) {
  PGW_REQUIRE(stream && exec_out, "pgw_graph_end: null argument");
  *exec_out = nullptr;
  hipGraph_t g = nullptr;
  if (hipStreamEndCapture(static_cast<hipStream_t>(stream), &g) != hipSuccess || !g) {
    (void)hipGetLastError();
    set_error("pgw_graph_end: hipStreamEndCapture failed (a launch in the capture failed?)");
    return PGW_ERR_HIP;
  }
  hipGraphExec_t ex = nullptr;
  const hipError_t rc = hipGraphInstantiate(&ex, g, nullptr, nullptr, 0);
  (void)hipGraphDestroy(g);
  if (rc != hipSuccess) {
    set_error("pgw_graph_end: hipGraphInstantiate failed");
    return PGW_ERR_HIP;
  }
  *exec_out = ex;
  return PGW_OK;
}

int32_t pgw_graph_launch(void* exec, void* stream) {
  PGW_REQUIRE(exec, "pgw_graph_launch: null graph");
  if (hipGraphLaunch(static_cast<hipGraphExec_t>(exec), static_cast<hipStream_t>(stream)) != hipSuccess) {
    set_error("pgw_graph_launch: hipGraphLaunch failed");
    return PGW_ERR_HIP;
  }
  return PGW_OK;
}

int32_t pgw_graph_destroy(void* exec) {
  if (exec) (void)hipGraphExecDestroy(static_cast<hipGraphExec_t>(exec));
  return PGW_OK;
}

}  // extern "C"

// Do-nothing rocprofiler-sdk tool for tools/startup_probe.py: T2_MODE=0 returns a
// configure result whose init does nothing; 1 creates a context; 2 also
// configures the dispatch counting service; 3 also starts the context.
#include <rocprofiler-sdk/registration.h>
#include <rocprofiler-sdk/rocprofiler.h>
#include <cstdlib>
#include <cstring>
namespace {
rocprofiler_context_id_t ctx{};
void dcb(rocprofiler_dispatch_counting_service_data_t, rocprofiler_counter_config_id_t*, rocprofiler_user_data_t*, void*) {}
void rcb(rocprofiler_dispatch_counting_service_data_t, rocprofiler_counter_record_t*, size_t, rocprofiler_user_data_t, void*) {}
int init(rocprofiler_client_finalize_t, void*) {
  const char* m = getenv("T2_MODE");
  int mode = m ? atoi(m) : 0;
  if (mode >= 1) rocprofiler_create_context(&ctx);
  if (mode >= 2) rocprofiler_configure_callback_dispatch_counting_service(ctx, dcb, nullptr, rcb, nullptr);
  if (mode >= 3) rocprofiler_start_context(ctx);
  return 0;
}
void fini(void*) {}
rocprofiler_tool_configure_result_t cfg = {sizeof(rocprofiler_tool_configure_result_t), init, fini, nullptr};
}
extern "C" rocprofiler_tool_configure_result_t* rocprofiler_configure(uint32_t, const char*, uint32_t, rocprofiler_client_id_t*) { return &cfg; }

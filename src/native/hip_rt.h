// The few HIP runtime entry points the native runtime needs, resolved with dlopen at first use so
// that _native.so loads (and the engine/storage work) on hosts without a GPU, and so that a process
// that never asks for device work never initialises HIP (data-loader parents fork workers).
#pragma once
#include <dlfcn.h>

#include <cstdint>
#include <mutex>

namespace mxamd {

struct HipRt {
  using IntFn = int (*)(int*);
  using SetDevFn = int (*)(int);
  using HostMallocFn = int (*)(void**, size_t, unsigned int);
  using PtrFn = int (*)(void*);
  using EventCreateFn = int (*)(void**, unsigned int);
  using EventRecordFn = int (*)(void*, void*);
  using StreamWaitFn = int (*)(void*, void*, unsigned int);
  using VoidFn = int (*)();

  IntFn get_device_count = nullptr;
  IntFn get_device = nullptr;
  SetDevFn set_device = nullptr;
  HostMallocFn host_malloc = nullptr;
  PtrFn host_free = nullptr;
  EventCreateFn event_create = nullptr;      // hipEventCreateWithFlags
  EventRecordFn event_record = nullptr;      // hipEventRecord(event, stream)
  StreamWaitFn stream_wait_event = nullptr;  // hipStreamWaitEvent(stream, event, 0)
  PtrFn event_synchronize = nullptr;
  PtrFn event_destroy = nullptr;
  VoidFn device_synchronize = nullptr;
  bool ok = false;         // runtime present and at least one device
  int num_devices = 0;

  static HipRt& Get() {
    static HipRt rt;
    static std::once_flag once;
    std::call_once(once, [] { rt.Load(); });
    return rt;
  }

 private:
  template <typename F>
  static void Sym(void* h, const char* name, F* out) {
    *out = reinterpret_cast<F>(dlsym(h, name));
  }
  void Load() {
    void* h = dlopen("libamdhip64.so", RTLD_LAZY | RTLD_LOCAL);
    if (!h) return;
    Sym(h, "hipGetDeviceCount", &get_device_count);
    Sym(h, "hipGetDevice", &get_device);
    Sym(h, "hipSetDevice", &set_device);
    Sym(h, "hipHostMalloc", &host_malloc);
    Sym(h, "hipHostFree", &host_free);
    Sym(h, "hipEventCreateWithFlags", &event_create);
    Sym(h, "hipEventRecord", &event_record);
    Sym(h, "hipStreamWaitEvent", &stream_wait_event);
    Sym(h, "hipEventSynchronize", &event_synchronize);
    Sym(h, "hipEventDestroy", &event_destroy);
    Sym(h, "hipDeviceSynchronize", &device_synchronize);
    int n = 0;
    ok = get_device_count && get_device && set_device && host_malloc && host_free && event_create &&
         event_record && stream_wait_event && event_synchronize && event_destroy && device_synchronize &&
         get_device_count(&n) == 0 && n > 0;
    num_devices = ok ? n : 0;
  }
};

}  // namespace mxamd

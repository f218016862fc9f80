// Dependency engine: asynchronous execution of operations with read/write
// dependencies on variables.
//
// Parity: src/engine/threaded_engine.{h,cc} (ThreadedVar / OprBlock /
// ThreadedEngine::Push / WaitForVar / WaitForAll) and naive_engine.cc.
//
// Design for an MI355X node.  Host operations (IO decode, checkpoint writes,
// kvstore bookkeeping, Python callbacks) run on a worker pool with per-variable
// reader/writer queues -- the reader/writer protocol of the reference's
// ThreadedVar.  A variable tracks
//   - the number of pending readers that have been granted access,
//   - whether a writer holds it,
//   - a FIFO of blocked operations,
//   - the HIP events of its last device writer and of the device readers since.
// Device operations (PushDevice, the ThreadedEnginePerDevice path of
// threaded_engine_perdevice.cc) are granted through the same queues but never
// block a worker on the GPU: when granted they make their stream wait on the
// events of their variables (hipStreamWaitEvent), enqueue their work on that
// stream, record one event and complete at once.  Ordering between device ops
// on different streams / devices is therefore enforced on the GPU; a host op
// whose variable was last written on a device synchronises on that event first.
//
// Debug mode (MXNET_ENGINE_DEBUG=1): every op checks, when it starts, that the
// versions of its variables are exactly the number of writes pushed before it
// and that no conflicting access is active; DebugAccess() lets code outside the
// engine declare a direct access so an undeclared concurrent use is reported.
#pragma once
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <exception>
#include <functional>
#include <memory>
#include <mutex>
#include <queue>
#include <string>
#include <thread>
#include <tuple>
#include <vector>

namespace mxamd {

struct Opr;

// A recorded HIP event (destroyed when the last holder drops it).
struct DevEvent {
  void* ev = nullptr;
  uintptr_t stream = 0;
  int device = -1;
  ~DevEvent();
};
using DevEventPtr = std::shared_ptr<DevEvent>;

struct Var {
  std::mutex mu;
  int num_pending_reads = 0;   // readers currently granted
  bool pending_write = false;  // a writer currently granted
  // blocked (op, is_write) in arrival order
  std::deque<std::pair<std::shared_ptr<Opr>, bool>> queue;
  std::exception_ptr exc;      // first exception raised by a writer of this var
  uint64_t version = 0;
  std::string name;
  DevEventPtr write_ev;                // last device writer
  std::vector<DevEventPtr> read_evs;   // device readers since that write
  // debug-mode bookkeeping
  uint64_t pushed_writes = 0;
  int active_readers = 0, active_writers = 0;
  // imperative dispatch on worker streams (Dispatcher): the slot / op sequence number of the last
  // dispatched writer (slot -1: written outside dispatch, i.e. on the caller's stream), the
  // (slot, seq) readers since that write, and the slots that already ordered themselves after the
  // caller's stream for an outside write in the current dispatch epoch
  int d_wslot = -1;
  uint64_t d_wseq = 0;
  std::vector<std::pair<int, uint64_t>> d_readers;
  uint64_t d_ext_epoch = 0;
  uint32_t d_ext_mask = 0;
};

using VarHandle = std::shared_ptr<Var>;
using Fn = std::function<void()>;

struct Opr {
  Fn fn;
  std::vector<VarHandle> const_vars;
  std::vector<VarHandle> mutable_vars;
  std::atomic<int> wait{0};
  int priority = 0;
  std::string name;
  uint64_t seq = 0;
  bool always_run = false;  // synchronisation ops run even if an input carries an exception
  // device ops
  bool is_device = false;
  uintptr_t stream = 0;
  int device = -1;
  // debug mode: expected version of each const / mutable var when the op starts
  std::vector<uint64_t> expect_const, expect_mut;
};

// Imperative operators on N streams per device (the ThreadedEnginePerDevice GPU workers of
// src/engine/threaded_engine_perdevice.cc, with the issue done inline by the calling thread: the
// operators are host-cheap kernel launches, so handing them to worker threads would only add
// latency).  Slot 0 is the caller's current stream, slots 1..N-1 are worker streams.  The dependency
// state lives on the engine variables of the arrays (Var::d_*):
//   * an operator runs on the slot that last wrote its first dispatched input (a chain stays on its
//     stream), else on the next slot round-robin;
//   * it waits on the GPU for writers of its inputs on other slots, and an in-place write also for
//     the other slots' readers of the target since its last write;
//   * inputs written outside dispatch (on the caller's stream) order a worker slot after the
//     caller's stream once per epoch;
//   * join() (every host-visible point) makes the caller's stream wait for all slots with work and
//     starts a new epoch.
// Cross-stream edges are HIP events recorded lazily: one event per slot is recorded only when a
// waiter needs it and no recorded event already covers the op it waits for.  With trace = true no
// HIP call is made and every wait edge is logged instead (CPU tests of the protocol).
class Dispatcher {
 public:
  explicit Dispatcher(bool trace) : trace_(trace) {}
  ~Dispatcher();
  void SetStreams(int device, const std::vector<uintptr_t>& workers);
  int Begin(int device, uintptr_t cur, const std::vector<VarHandle>& reads);
  void Write(int device, uintptr_t cur, int slot, const VarHandle& target);
  void End(int device, int slot, const std::vector<VarHandle>& reads, const std::vector<VarHandle>& writes);
  // returns the slots joined
  std::vector<int> Join(int device, uintptr_t cur);
  static int SlotOf(const VarHandle& v);
  std::vector<std::tuple<int, int, int>> TakeTrace();
  uint64_t waits() const { return waits_; }

 private:
  struct Slot {
    uintptr_t stream = 0;
    uint64_t seq = 0;       // operators issued on this slot
    uint64_t rec_seq = 0;   // ops covered by the last recorded event
    void* ev = nullptr;
    bool has_ev = false;
  };
  struct Dev {
    std::vector<Slot> slots;   // [0] = the caller's stream (handle passed per call)
    uint32_t dirty = 0;
    int rr = 0;
  };
  Dev& D(int device);
  void WaitFor(int device, Dev& d, int waiter, uintptr_t cur, int on, uint64_t seq);
  uintptr_t StreamOf(Dev& d, int slot, uintptr_t cur) { return slot == 0 ? cur : d.slots[slot].stream; }

  bool trace_;
  std::mutex mu_;
  std::vector<Dev> devs_;
  uint64_t epoch_ = 1;
  uint64_t waits_ = 0;
  std::vector<std::tuple<int, int, int>> log_;
};

class Engine {
 public:
  explicit Engine(int num_workers, bool naive, bool debug = false);
  ~Engine();
  VarHandle NewVar(const std::string& name = "");
  void Push(Fn fn, const std::vector<VarHandle>& const_vars,
            const std::vector<VarHandle>& mutable_vars, int priority,
            const std::string& name, bool always_run = false);
  // Device op: `launch` enqueues work on `stream` (a hipStream_t) of `device`.
  void PushDevice(Fn launch, const std::vector<VarHandle>& const_vars,
                  const std::vector<VarHandle>& mutable_vars, uintptr_t stream, int device,
                  int priority, const std::string& name);
  void WaitForVar(const VarHandle& v);
  // Make `stream` wait (on the GPU) for the device write of `v`: blocks the caller only until the ops
  // pushed on `v` so far have been *issued*, never on GPU execution.
  // A pending exception of `v` is rethrown here once and cleared (WaitForVar semantics).
  void StreamWaitVar(const VarHandle& v, uintptr_t stream, int device);
  // Drop a pending exception of `v` that was reported elsewhere (e.g. a shared ordering variable
  // whose failing op's error already reached the caller through an output variable).
  void ClearException(const VarHandle& v);
  // Debug mode: declare a direct (non-engine) access; a conflicting active engine access is a race.
  void DebugAccess(const VarHandle& v, bool write);
  bool debug() const { return debug_; }
  uint64_t violations() const { return violations_.load(); }
  std::string last_violation();
  uint64_t device_ops() const { return device_ops_.load(); }
  void WaitForAll();
  int64_t Pending() const { return pending_.load(); }
  bool naive() const { return naive_; }
  int num_workers() const { return static_cast<int>(workers_.size()); }
  // statistics
  uint64_t executed() const { return executed_.load(); }

 private:
  void PushOp(std::shared_ptr<Opr> op, const std::vector<VarHandle>& const_vars,
              const std::vector<VarHandle>& mutable_vars);
  void Dispatch(std::shared_ptr<Opr> op);
  void RunDevice(const std::shared_ptr<Opr>& op);
  void SyncHost(const std::shared_ptr<Opr>& op);
  std::exception_ptr DebugBegin(const std::shared_ptr<Opr>& op);
  void DebugEnd(const std::shared_ptr<Opr>& op);
  void Violation(const std::string& msg);
  void Execute(std::shared_ptr<Opr> op);
  void Complete(const std::shared_ptr<Opr>& op, std::exception_ptr exc);
  bool AppendRead(const VarHandle& v, const std::shared_ptr<Opr>& op);
  bool AppendWrite(const VarHandle& v, const std::shared_ptr<Opr>& op);
  void ReleaseRead(const VarHandle& v);
  void ReleaseWrite(const VarHandle& v, std::exception_ptr exc);
  void WorkerLoop();

  struct Cmp {
    bool operator()(const std::shared_ptr<Opr>& a, const std::shared_ptr<Opr>& b) const {
      if (a->priority != b->priority) return a->priority < b->priority;
      return a->seq > b->seq;  // FIFO among equal priorities
    }
  };

  bool naive_;
  bool debug_;
  std::atomic<uint64_t> violations_{0};
  std::atomic<uint64_t> device_ops_{0};
  std::mutex vmu_;
  std::string last_violation_;
  std::mutex devmu_;
  std::vector<int> devices_used_;
  std::atomic<bool> stop_{false};
  std::atomic<int64_t> pending_{0};
  std::atomic<uint64_t> executed_{0};
  std::atomic<uint64_t> seq_{0};
  std::mutex qmu_;
  std::condition_variable qcv_;
  std::priority_queue<std::shared_ptr<Opr>, std::vector<std::shared_ptr<Opr>>, Cmp> ready_;
  std::mutex allmu_;
  std::condition_variable allcv_;
  std::vector<std::thread> workers_;
  std::mutex excmu_;
  std::exception_ptr global_exc_;
};

}  // namespace mxamd

// Dependency engine: asynchronous execution of operations with read/write
// dependencies on variables.
//
// Parity: src/engine/threaded_engine.{h,cc} (ThreadedVar / OprBlock /
// ThreadedEngine::Push / WaitForVar / WaitForAll) and naive_engine.cc.
//
// Design for an MI355X node: device work is already ordered by HIP streams,
// so this engine schedules the *host-side* work around it (IO decode,
// checkpoint writes, kvstore bookkeeping, Python callbacks) on a worker pool
// with per-variable reader/writer queues.  A variable tracks
//   - the number of pending readers that have been granted access,
//   - whether a writer holds it,
//   - a FIFO of blocked operations,
// exactly the reader/writer protocol of the reference's ThreadedVar.
#pragma once
#include <atomic>
#include <condition_variable>
#include <deque>
#include <exception>
#include <functional>
#include <memory>
#include <mutex>
#include <queue>
#include <string>
#include <thread>
#include <vector>

namespace mxamd {

struct Opr;

struct Var {
  std::mutex mu;
  int num_pending_reads = 0;   // readers currently granted
  bool pending_write = false;  // a writer currently granted
  // blocked (op, is_write) in arrival order
  std::deque<std::pair<std::shared_ptr<Opr>, bool>> queue;
  std::exception_ptr exc;      // first exception raised by a writer of this var
  uint64_t version = 0;
  std::string name;
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
};

class Engine {
 public:
  explicit Engine(int num_workers, bool naive);
  ~Engine();
  VarHandle NewVar(const std::string& name = "");
  void Push(Fn fn, const std::vector<VarHandle>& const_vars,
            const std::vector<VarHandle>& mutable_vars, int priority,
            const std::string& name, bool always_run = false);
  void WaitForVar(const VarHandle& v);
  void WaitForAll();
  int64_t Pending() const { return pending_.load(); }
  bool naive() const { return naive_; }
  int num_workers() const { return static_cast<int>(workers_.size()); }
  // statistics
  uint64_t executed() const { return executed_.load(); }

 private:
  void Dispatch(std::shared_ptr<Opr> op);
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

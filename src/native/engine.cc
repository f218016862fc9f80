// Threaded dependency engine (see engine.h for the protocol).
#include "engine.h"

#include <algorithm>
#include <stdexcept>

#include "hip_rt.h"

namespace mxamd {

DevEvent::~DevEvent() {
  if (ev) HipRt::Get().event_destroy(ev);
}

namespace {

void HipCheck(int rc, const char* what) {
  if (rc != 0) throw std::runtime_error(std::string("engine device op: ") + what + " failed (hip error " +
                                        std::to_string(rc) + ")");
}

}  // namespace

Engine::Engine(int num_workers, bool naive, bool debug) : naive_(naive), debug_(debug) {
  if (!naive_) {
    if (num_workers <= 0) num_workers = 1;
    for (int i = 0; i < num_workers; ++i) workers_.emplace_back([this] { WorkerLoop(); });
  }
}

Engine::~Engine() {
  {
    std::lock_guard<std::mutex> lk(qmu_);
    stop_ = true;
  }
  qcv_.notify_all();
  for (auto& t : workers_) t.join();
}

VarHandle Engine::NewVar(const std::string& name) {
  auto v = std::make_shared<Var>();
  v->name = name;
  return v;
}

bool Engine::AppendRead(const VarHandle& v, const std::shared_ptr<Opr>& op) {
  std::lock_guard<std::mutex> lk(v->mu);
  if (!v->pending_write && v->queue.empty()) {
    ++v->num_pending_reads;
    return true;
  }
  v->queue.emplace_back(op, false);
  return false;
}

bool Engine::AppendWrite(const VarHandle& v, const std::shared_ptr<Opr>& op) {
  std::lock_guard<std::mutex> lk(v->mu);
  if (!v->pending_write && v->num_pending_reads == 0 && v->queue.empty()) {
    v->pending_write = true;
    return true;
  }
  v->queue.emplace_back(op, true);
  return false;
}

void Engine::PushOp(std::shared_ptr<Opr> op, const std::vector<VarHandle>& const_vars,
                    const std::vector<VarHandle>& mutable_vars) {
  op->mutable_vars = mutable_vars;
  // a variable that is both read and written is only written
  for (const auto& v : const_vars) {
    if (std::find(mutable_vars.begin(), mutable_vars.end(), v) == mutable_vars.end() &&
        std::find(op->const_vars.begin(), op->const_vars.end(), v) == op->const_vars.end())
      op->const_vars.push_back(v);
  }
  op->seq = seq_.fetch_add(1);
  if (debug_) {
    // the version a var must have when this op starts = writes pushed before it
    for (const auto& v : op->const_vars) {
      std::lock_guard<std::mutex> lk(v->mu);
      op->expect_const.push_back(v->pushed_writes);
    }
    for (const auto& v : op->mutable_vars) {
      std::lock_guard<std::mutex> lk(v->mu);
      op->expect_mut.push_back(v->pushed_writes++);
    }
  }
  ++pending_;
  if (naive_) {
    Execute(op);
    return;
  }
  op->wait = static_cast<int>(op->const_vars.size() + op->mutable_vars.size()) + 1;
  int granted = 0;
  for (const auto& v : op->const_vars) granted += AppendRead(v, op) ? 1 : 0;
  for (const auto& v : op->mutable_vars) granted += AppendWrite(v, op) ? 1 : 0;
  if (op->wait.fetch_sub(granted + 1) == granted + 1) Dispatch(op);
}

void Engine::Push(Fn fn, const std::vector<VarHandle>& const_vars,
                  const std::vector<VarHandle>& mutable_vars, int priority,
                  const std::string& name, bool always_run) {
  auto op = std::make_shared<Opr>();
  op->fn = std::move(fn);
  op->always_run = always_run;
  op->priority = priority;
  op->name = name;
  PushOp(std::move(op), const_vars, mutable_vars);
}

void Engine::PushDevice(Fn launch, const std::vector<VarHandle>& const_vars,
                        const std::vector<VarHandle>& mutable_vars, uintptr_t stream, int device,
                        int priority, const std::string& name) {
  auto op = std::make_shared<Opr>();
  op->fn = std::move(launch);
  op->priority = priority;
  op->name = name;
  op->is_device = true;
  op->stream = stream;
  op->device = device;
  PushOp(std::move(op), const_vars, mutable_vars);
}

void Engine::Dispatch(std::shared_ptr<Opr> op) {
  {
    std::lock_guard<std::mutex> lk(qmu_);
    ready_.push(std::move(op));
  }
  qcv_.notify_one();
}

void Engine::WorkerLoop() {
  for (;;) {
    std::shared_ptr<Opr> op;
    {
      std::unique_lock<std::mutex> lk(qmu_);
      qcv_.wait(lk, [this] { return stop_ || !ready_.empty(); });
      if (stop_ && ready_.empty()) return;
      op = ready_.top();
      ready_.pop();
    }
    Execute(op);
  }
}

// Device op body: stream waits on the events of its vars, launch, one event recorded for all of them.
void Engine::RunDevice(const std::shared_ptr<Opr>& op) {
  HipRt& rt = HipRt::Get();
  if (!rt.ok) {       // no GPU runtime: the launch runs as a plain host op (CPU tensors)
    if (op->fn) op->fn();
    return;
  }
  int prev = -1;
  HipCheck(rt.get_device(&prev), "hipGetDevice");
  if (op->device >= 0 && op->device != prev) HipCheck(rt.set_device(op->device), "hipSetDevice");
  std::vector<DevEventPtr> waits;
  for (const auto& v : op->const_vars) {
    std::lock_guard<std::mutex> lk(v->mu);
    if (v->write_ev) waits.push_back(v->write_ev);
  }
  for (const auto& v : op->mutable_vars) {
    std::lock_guard<std::mutex> lk(v->mu);
    if (v->write_ev) waits.push_back(v->write_ev);
    waits.insert(waits.end(), v->read_evs.begin(), v->read_evs.end());
  }
  for (const auto& e : waits)
    if (e->stream != op->stream || e->device != op->device)   // same stream: already ordered
      HipCheck(rt.stream_wait_event(reinterpret_cast<void*>(op->stream), e->ev, 0), "hipStreamWaitEvent");
  try {
    if (op->fn) op->fn();
  } catch (...) {
    if (op->device >= 0 && op->device != prev) rt.set_device(prev);
    throw;
  }
  auto ev = std::make_shared<DevEvent>();
  ev->stream = op->stream;
  ev->device = op->device;
  HipCheck(rt.event_create(&ev->ev, 0x2 /* hipEventDisableTiming */), "hipEventCreateWithFlags");
  HipCheck(rt.event_record(ev->ev, reinterpret_cast<void*>(op->stream)), "hipEventRecord");
  if (op->device >= 0 && op->device != prev) rt.set_device(prev);
  for (const auto& v : op->const_vars) {
    std::lock_guard<std::mutex> lk(v->mu);
    // one read event per (device, stream): a later event on the same stream implies the earlier ones,
    // so a read-only variable (weights at inference) keeps a bounded list
    auto& r = v->read_evs;
    r.erase(std::remove_if(r.begin(), r.end(),
                           [&](const DevEventPtr& e) { return e->stream == ev->stream && e->device == ev->device; }),
            r.end());
    r.push_back(ev);
  }
  for (const auto& v : op->mutable_vars) {
    std::lock_guard<std::mutex> lk(v->mu);
    v->write_ev = ev;
    v->read_evs.clear();
  }
  {
    std::lock_guard<std::mutex> lk(devmu_);
    if (std::find(devices_used_.begin(), devices_used_.end(), op->device) == devices_used_.end())
      devices_used_.push_back(op->device);
  }
  ++device_ops_;
}

// Host op body prologue: data last written (or read, for a writer) on a device must be complete.
void Engine::SyncHost(const std::shared_ptr<Opr>& op) {
  std::vector<DevEventPtr> waits;
  for (const auto& v : op->const_vars) {
    std::lock_guard<std::mutex> lk(v->mu);
    if (v->write_ev) waits.push_back(v->write_ev);
  }
  for (const auto& v : op->mutable_vars) {
    std::lock_guard<std::mutex> lk(v->mu);
    if (v->write_ev) waits.push_back(v->write_ev);
    waits.insert(waits.end(), v->read_evs.begin(), v->read_evs.end());
  }
  for (const auto& e : waits) HipCheck(HipRt::Get().event_synchronize(e->ev), "hipEventSynchronize");
}

void Engine::Violation(const std::string& msg) {
  ++violations_;
  std::lock_guard<std::mutex> lk(vmu_);
  last_violation_ = msg;
}

std::string Engine::last_violation() {
  std::lock_guard<std::mutex> lk(vmu_);
  return last_violation_;
}

std::exception_ptr Engine::DebugBegin(const std::shared_ptr<Opr>& op) {
  std::string err;
  for (size_t i = 0; i < op->const_vars.size(); ++i) {
    const auto& v = op->const_vars[i];
    std::lock_guard<std::mutex> lk(v->mu);
    if (v->version != op->expect_const[i] || v->active_writers != 0)
      err = "read of var '" + v->name + "' by op '" + op->name + "' at version " + std::to_string(v->version) +
            " (expected " + std::to_string(op->expect_const[i]) + ", active writers " +
            std::to_string(v->active_writers) + ")";
    ++v->active_readers;
  }
  for (size_t i = 0; i < op->mutable_vars.size(); ++i) {
    const auto& v = op->mutable_vars[i];
    std::lock_guard<std::mutex> lk(v->mu);
    if (v->version != op->expect_mut[i] || v->active_writers != 0 || v->active_readers != 0)
      err = "write of var '" + v->name + "' by op '" + op->name + "' at version " + std::to_string(v->version) +
            " (expected " + std::to_string(op->expect_mut[i]) + ", active readers " +
            std::to_string(v->active_readers) + ", writers " + std::to_string(v->active_writers) + ")";
    ++v->active_writers;
  }
  if (err.empty()) return nullptr;
  Violation("engine race: " + err);
  return std::make_exception_ptr(std::runtime_error("engine race: " + err));
}

void Engine::DebugEnd(const std::shared_ptr<Opr>& op) {
  for (const auto& v : op->const_vars) {
    std::lock_guard<std::mutex> lk(v->mu);
    --v->active_readers;
  }
  for (const auto& v : op->mutable_vars) {
    std::lock_guard<std::mutex> lk(v->mu);
    --v->active_writers;
  }
}

void Engine::DebugAccess(const VarHandle& v, bool write) {
  if (!debug_) return;
  std::lock_guard<std::mutex> lk(v->mu);
  if (v->active_writers != 0 || (write && v->active_readers != 0))
    Violation("engine race: direct " + std::string(write ? "write" : "read") + " of var '" + v->name +
              "' while an engine op holds it (readers " + std::to_string(v->active_readers) + ", writers " +
              std::to_string(v->active_writers) + ")");
}

void Engine::Execute(std::shared_ptr<Opr> op) {
  std::exception_ptr exc;
  std::exception_ptr race = debug_ && !op->always_run ? DebugBegin(op) : nullptr;
  if (op->always_run) {
    if (op->fn) op->fn();
    ++executed_;
    if (naive_) {
      if (--pending_ == 0) {
        std::lock_guard<std::mutex> lk(allmu_);
        allcv_.notify_all();
      }
      return;
    }
    Complete(op, nullptr);
    return;
  }
  // exception propagation: an input written by a failed op poisons this op
  for (const auto& v : op->const_vars) {
    std::lock_guard<std::mutex> lk(v->mu);
    if (v->exc) { exc = v->exc; break; }
  }
  if (!exc) {
    for (const auto& v : op->mutable_vars) {
      std::lock_guard<std::mutex> lk(v->mu);
      if (v->exc) { exc = v->exc; break; }
    }
  }
  if (!exc && race) exc = race;
  if (!exc) {
    try {
      if (op->is_device) {
        RunDevice(op);
      } else {
        SyncHost(op);
        if (op->fn) op->fn();
      }
    } catch (...) {
      exc = std::current_exception();
    }
  }
  if (debug_) DebugEnd(op);
  ++executed_;
  if (naive_) {
    for (const auto& v : op->mutable_vars) {
      std::lock_guard<std::mutex> lk(v->mu);
      ++v->version;
      if (exc) v->exc = exc;
    }
    if (exc) {
      std::lock_guard<std::mutex> lk(excmu_);
      if (!global_exc_) global_exc_ = exc;
    }
    if (--pending_ == 0) {
      std::lock_guard<std::mutex> lk(allmu_);
      allcv_.notify_all();
    }
    return;
  }
  Complete(op, exc);
}

void Engine::ReleaseRead(const VarHandle& v) {
  std::shared_ptr<Opr> next;
  {
    std::lock_guard<std::mutex> lk(v->mu);
    --v->num_pending_reads;
    if (v->num_pending_reads == 0 && !v->queue.empty() && v->queue.front().second) {
      next = v->queue.front().first;
      v->queue.pop_front();
      v->pending_write = true;
    }
  }
  if (next && next->wait.fetch_sub(1) == 1) Dispatch(next);
}

void Engine::ReleaseWrite(const VarHandle& v, std::exception_ptr exc) {
  std::vector<std::shared_ptr<Opr>> granted;
  {
    std::lock_guard<std::mutex> lk(v->mu);
    v->pending_write = false;
    ++v->version;
    if (exc && !v->exc) v->exc = exc;
    while (!v->queue.empty()) {
      auto& front = v->queue.front();
      if (front.second) {  // writer
        if (v->num_pending_reads == 0 && granted.empty()) {
          v->pending_write = true;
          granted.push_back(front.first);
          v->queue.pop_front();
        }
        break;
      }
      ++v->num_pending_reads;
      granted.push_back(front.first);
      v->queue.pop_front();
    }
  }
  for (auto& op : granted)
    if (op->wait.fetch_sub(1) == 1) Dispatch(op);
}

void Engine::Complete(const std::shared_ptr<Opr>& op, std::exception_ptr exc) {
  if (exc) {
    std::lock_guard<std::mutex> lk(excmu_);
    if (!global_exc_) global_exc_ = exc;
  }
  for (const auto& v : op->const_vars) ReleaseRead(v);
  for (const auto& v : op->mutable_vars) ReleaseWrite(v, exc);
  if (--pending_ == 0) {
    std::lock_guard<std::mutex> lk(allmu_);
    allcv_.notify_all();
  }
}

void Engine::WaitForVar(const VarHandle& v) {
  auto done = std::make_shared<std::pair<std::mutex, std::condition_variable>>();
  auto flag = std::make_shared<bool>(false);
  Push([done, flag] {
         std::lock_guard<std::mutex> lk(done->first);
         *flag = true;
         done->second.notify_all();
       },
       {v}, {}, 1 << 20, "WaitForVar", /*always_run=*/true);
  {
    std::unique_lock<std::mutex> lk(done->first);
    done->second.wait(lk, [&] { return *flag; });
  }
  std::exception_ptr exc;
  DevEventPtr ev;
  {
    std::lock_guard<std::mutex> lk(v->mu);
    exc = v->exc;
    v->exc = nullptr;
    ev = v->write_ev;
  }
  if (ev) HipCheck(HipRt::Get().event_synchronize(ev->ev), "hipEventSynchronize");   // the device write too
  if (exc) {
    std::lock_guard<std::mutex> lk(excmu_);
    if (global_exc_ == exc) global_exc_ = nullptr;
    std::rethrow_exception(exc);
  }
}

void Engine::StreamWaitVar(const VarHandle& v, uintptr_t stream, int device) {
  auto done = std::make_shared<std::pair<std::mutex, std::condition_variable>>();
  auto flag = std::make_shared<bool>(false);
  Push([done, flag] {
         std::lock_guard<std::mutex> lk(done->first);
         *flag = true;
         done->second.notify_all();
       },
       {v}, {}, 1 << 20, "StreamWaitVar", /*always_run=*/true);
  {
    std::unique_lock<std::mutex> lk(done->first);
    done->second.wait(lk, [&] { return *flag; });
  }
  DevEventPtr ev;
  std::exception_ptr exc;
  {
    std::lock_guard<std::mutex> lk(v->mu);
    ev = v->write_ev;
    exc = v->exc;
    v->exc = nullptr;   // reported here, like WaitForVar: later ops on v run again
  }
  if (exc) {
    std::lock_guard<std::mutex> lk(excmu_);
    if (global_exc_ == exc) global_exc_ = nullptr;
    std::rethrow_exception(exc);
  }
  if (!ev || (ev->stream == stream && ev->device == device)) return;
  HipRt& rt = HipRt::Get();
  int prev = -1;
  HipCheck(rt.get_device(&prev), "hipGetDevice");
  if (device >= 0 && device != prev) HipCheck(rt.set_device(device), "hipSetDevice");
  const int rc = rt.stream_wait_event(reinterpret_cast<void*>(stream), ev->ev, 0);
  if (device >= 0 && device != prev) rt.set_device(prev);
  HipCheck(rc, "hipStreamWaitEvent");
}

void Engine::ClearException(const VarHandle& v) {
  std::exception_ptr exc;
  {
    std::lock_guard<std::mutex> lk(v->mu);
    exc = v->exc;
    v->exc = nullptr;
  }
  if (exc) {
    std::lock_guard<std::mutex> lk(excmu_);
    if (global_exc_ == exc) global_exc_ = nullptr;
  }
}

void Engine::WaitForAll() {
  {
    std::unique_lock<std::mutex> lk(allmu_);
    allcv_.wait(lk, [this] { return pending_.load() == 0; });
  }
  std::vector<int> devs;
  {
    std::lock_guard<std::mutex> lk(devmu_);
    devs = devices_used_;
  }
  if (!devs.empty()) {
    HipRt& rt = HipRt::Get();
    int prev = -1;
    HipCheck(rt.get_device(&prev), "hipGetDevice");
    for (int d : devs) {
      if (d >= 0) HipCheck(rt.set_device(d), "hipSetDevice");
      HipCheck(rt.device_synchronize(), "hipDeviceSynchronize");
    }
    rt.set_device(prev);
  }
  std::exception_ptr exc;
  {
    std::lock_guard<std::mutex> lk(excmu_);
    exc = global_exc_;
    global_exc_ = nullptr;
  }
  if (exc) std::rethrow_exception(exc);
}

// ------------------------------------------------------------------ imperative dispatch (engine.h)
Dispatcher::~Dispatcher() {
  if (trace_) return;
  for (auto& d : devs_)
    for (auto& sl : d.slots)
      if (sl.ev) HipRt::Get().event_destroy(sl.ev);
}

Dispatcher::Dev& Dispatcher::D(int device) {
  if (device < 0) throw std::runtime_error("dispatcher: bad device");
  if (static_cast<int>(devs_.size()) <= device) devs_.resize(device + 1);
  Dev& d = devs_[device];
  if (d.slots.empty()) d.slots.resize(1);
  return d;
}

void Dispatcher::SetStreams(int device, const std::vector<uintptr_t>& workers) {
  std::lock_guard<std::mutex> lk(mu_);
  Dev& d = D(device);
  if (workers.size() + 1 > 32) throw std::runtime_error("dispatcher: at most 32 slots per device");
  d.slots.resize(workers.size() + 1);
  for (size_t i = 0; i < workers.size(); ++i) d.slots[i + 1].stream = workers[i];
  if (d.rr >= static_cast<int>(d.slots.size())) d.rr = 0;
}

// make slot `waiter` wait for slot `on`'s operators up to `seq` (seq 0: everything issued so far)
void Dispatcher::WaitFor(int device, Dev& d, int waiter, uintptr_t cur, int on, uint64_t seq) {
  if (waiter == on) return;
  Slot& src = d.slots[on];
  const uint64_t need = seq ? seq : src.seq;
  ++waits_;
  if (trace_) {
    log_.emplace_back(device, waiter, on);
    return;
  }
  HipRt& rt = HipRt::Get();
  if (!src.has_ev || src.rec_seq < need || on == 0) {
    // slot 0 is the caller's stream: outside writes are not counted, so its event is always fresh
    if (!src.ev) HipCheck(rt.event_create(&src.ev, 0x2 /* hipEventDisableTiming */), "hipEventCreateWithFlags");
    HipCheck(rt.event_record(src.ev, reinterpret_cast<void*>(StreamOf(d, on, cur))), "hipEventRecord");
    src.has_ev = true;
    src.rec_seq = src.seq;
  }
  HipCheck(rt.stream_wait_event(reinterpret_cast<void*>(StreamOf(d, waiter, cur)), src.ev, 0),
           "hipStreamWaitEvent");
}

int Dispatcher::Begin(int device, uintptr_t cur, const std::vector<VarHandle>& reads) {
  std::lock_guard<std::mutex> lk(mu_);
  Dev& d = D(device);
  const int ns = static_cast<int>(d.slots.size());
  int slot = -1;
  for (const auto& v : reads) {
    std::lock_guard<std::mutex> vl(v->mu);
    if (v->d_wslot >= 0 && v->d_wslot < ns) {
      slot = v->d_wslot;
      break;
    }
  }
  if (slot < 0) {
    slot = d.rr;
    d.rr = (d.rr + 1) % ns;
  }
  // one wait per source slot: the newest op it must cover (0 = everything issued so far)
  std::vector<int64_t> need(ns, -1);
  auto want = [&](int on, uint64_t q) {
    if (on == slot) return;
    if (need[on] < 0 || q == 0 || (need[on] != 0 && static_cast<int64_t>(q) > need[on])) need[on] = static_cast<int64_t>(q);
  };
  for (const auto& v : reads) {
    std::lock_guard<std::mutex> vl(v->mu);
    if (v->d_wslot >= 0 && v->d_wslot < ns) {
      want(v->d_wslot, v->d_wseq);
      continue;
    }
    // written on the caller's stream: a worker slot orders after it once per epoch
    if (slot == 0) continue;
    if (v->d_ext_epoch != epoch_) {
      v->d_ext_epoch = epoch_;
      v->d_ext_mask = 0;
    }
    if (v->d_ext_mask & (1u << slot)) continue;
    v->d_ext_mask |= 1u << slot;
    want(0, 0);
  }
  for (int on = 0; on < ns; ++on)
    if (need[on] >= 0) WaitFor(device, d, slot, cur, on, static_cast<uint64_t>(need[on]));
  return slot;
}

void Dispatcher::Write(int device, uintptr_t cur, int slot, const VarHandle& v) {
  std::lock_guard<std::mutex> lk(mu_);
  Dev& d = D(device);
  const int ns = static_cast<int>(d.slots.size());
  std::vector<int64_t> need(ns, -1);
  auto want = [&](int on, uint64_t q) {
    if (on == slot) return;
    if (need[on] < 0 || q == 0 || (need[on] != 0 && static_cast<int64_t>(q) > need[on])) need[on] = static_cast<int64_t>(q);
  };
  {
    std::lock_guard<std::mutex> vl(v->mu);
    if (v->d_wslot >= 0 && v->d_wslot < ns) want(v->d_wslot, v->d_wseq);
    else want(0, 0);
    for (const auto& r : v->d_readers)
      if (r.first < ns) want(r.first, r.second);
  }
  for (int on = 0; on < ns; ++on)
    if (need[on] >= 0) WaitFor(device, d, slot, cur, on, static_cast<uint64_t>(need[on]));
}

void Dispatcher::End(int device, int slot, const std::vector<VarHandle>& reads, const std::vector<VarHandle>& writes) {
  std::lock_guard<std::mutex> lk(mu_);
  Dev& d = D(device);
  const uint64_t seq = ++d.slots[slot].seq;
  if (slot) d.dirty |= 1u << slot;
  for (const auto& v : reads) {
    std::lock_guard<std::mutex> vl(v->mu);
    bool found = false;
    for (auto& r : v->d_readers)
      if (r.first == slot) {
        r.second = seq;
        found = true;
      }
    if (!found) v->d_readers.emplace_back(slot, seq);
  }
  for (const auto& v : writes) {
    std::lock_guard<std::mutex> vl(v->mu);
    v->d_wslot = slot;
    v->d_wseq = seq;
    v->d_readers.clear();
  }
}

std::vector<int> Dispatcher::Join(int device, uintptr_t cur) {
  std::lock_guard<std::mutex> lk(mu_);
  ++epoch_;
  std::vector<int> joined;
  if (device < 0 || device >= static_cast<int>(devs_.size())) return joined;
  Dev& d = devs_[device];
  for (int s = 1; s < static_cast<int>(d.slots.size()); ++s) {
    if (!(d.dirty & (1u << s))) continue;
    WaitFor(device, d, 0, cur, s, 0);
    joined.push_back(s);
  }
  d.dirty = 0;
  return joined;
}

int Dispatcher::SlotOf(const VarHandle& v) {
  std::lock_guard<std::mutex> vl(v->mu);
  return v->d_wslot;
}

std::vector<std::tuple<int, int, int>> Dispatcher::TakeTrace() {
  std::lock_guard<std::mutex> lk(mu_);
  std::vector<std::tuple<int, int, int>> out;
  out.swap(log_);
  return out;
}

}  // namespace mxamd

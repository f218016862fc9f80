// Threaded dependency engine (see engine.h for the protocol).
#include "engine.h"

#include <algorithm>

namespace mxamd {

Engine::Engine(int num_workers, bool naive) : naive_(naive) {
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

void Engine::Push(Fn fn, const std::vector<VarHandle>& const_vars,
                  const std::vector<VarHandle>& mutable_vars, int priority,
                  const std::string& name, bool always_run) {
  auto op = std::make_shared<Opr>();
  op->fn = std::move(fn);
  op->always_run = always_run;
  op->mutable_vars = mutable_vars;
  // a variable that is both read and written is only written
  for (const auto& v : const_vars) {
    if (std::find(mutable_vars.begin(), mutable_vars.end(), v) == mutable_vars.end() &&
        std::find(op->const_vars.begin(), op->const_vars.end(), v) == op->const_vars.end())
      op->const_vars.push_back(v);
  }
  op->priority = priority;
  op->name = name;
  op->seq = seq_.fetch_add(1);
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

void Engine::Execute(std::shared_ptr<Opr> op) {
  std::exception_ptr exc;
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
  if (!exc) {
    try {
      if (op->fn) op->fn();
    } catch (...) {
      exc = std::current_exception();
    }
  }
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
  {
    std::lock_guard<std::mutex> lk(v->mu);
    exc = v->exc;
    v->exc = nullptr;
  }
  if (exc) {
    std::lock_guard<std::mutex> lk(excmu_);
    if (global_exc_ == exc) global_exc_ = nullptr;
    std::rethrow_exception(exc);
  }
}

void Engine::WaitForAll() {
  {
    std::unique_lock<std::mutex> lk(allmu_);
    allcv_.wait(lk, [this] { return pending_.load() == 0; });
  }
  std::exception_ptr exc;
  {
    std::lock_guard<std::mutex> lk(excmu_);
    exc = global_exc_;
    global_exc_ = nullptr;
  }
  if (exc) std::rethrow_exception(exc);
}

}  // namespace mxamd

// Host-side fork/join helper for the CPU work around the device path (metrics, test
// scores, text parsing and formatting).  Same interface as the reference's
// ParallelExecutor (qmf/utils/ParallelExecutor.h:28-65): execute() hands task ids to
// threads with a stride, mapReduce() folds per thread and then over threads in order.
// Threads are started per call: these are coarse, infrequent jobs.
#pragma once

#include <algorithm>
#include <cstddef>
#include <functional>
#include <thread>
#include <vector>

namespace qmf {

class ParallelExecutor {
 public:
  explicit ParallelExecutor(const size_t nthreads) : nthreads_(std::max<size_t>(1, nthreads)) {}

  size_t nthreads() const { return nthreads_; }

  // func(taskId) for taskId in [0, ntasks)
  template <typename FuncT>
  void execute(const size_t ntasks, FuncT&& func) {
    const size_t nt = std::min(nthreads_, std::max<size_t>(ntasks, 1));
    run(nt, [&](const size_t t) {
      for (size_t task = t; task < ntasks; task += nt) func(task);
    });
  }

  // reducer(... reducer(neutral, mapper(t0)) ...) per thread, then over threads in order
  template <typename T, typename MapperT, typename ReducerT>
  T mapReduce(const size_t ntasks, MapperT&& mapper, ReducerT&& reducer, T neutral) {
    const size_t nt = std::min(nthreads_, std::max<size_t>(ntasks, 1));
    std::vector<T> part(nt, neutral);
    run(nt, [&](const size_t t) {
      T acc = neutral;
      for (size_t task = t; task < ntasks; task += nt) acc = reducer(acc, mapper(task));
      part[t] = acc;
    });
    T res = neutral;
    for (const T& p : part) res = reducer(res, p);
    return res;
  }

  // mapper over every element (contiguous blocks per thread, all elements included)
  template <typename T, typename ElemT, typename MapperT, typename ReducerT>
  T mapReduce(const std::vector<ElemT>& elems, MapperT&& mapper, ReducerT&& reducer,
              T neutral) {
    const size_t n = elems.size();
    const size_t nt = std::min(nthreads_, std::max<size_t>(n, 1));
    std::vector<T> part(nt, neutral);
    run(nt, [&](const size_t t) {
      T acc = neutral;
      const size_t b = n * t / nt, e = n * (t + 1) / nt;
      for (size_t i = b; i < e; ++i) acc = reducer(acc, mapper(elems[i]));
      part[t] = acc;
    });
    T res = neutral;
    for (const T& p : part) res = reducer(res, p);
    return res;
  }

  // body(t) on nt threads (t = 0 runs on the caller)
  template <typename BodyT>
  static void run(const size_t nt, BodyT&& body) {
    std::vector<std::thread> th;
    th.reserve(nt > 0 ? nt - 1 : 0);
    for (size_t t = 1; t < nt; ++t) th.emplace_back([&body, t] { body(t); });
    if (nt > 0) body(0);
    for (auto& x : th) x.join();
  }

 private:
  size_t nthreads_;
};

}  // namespace qmf

// RAII handle on a qmfx device context (include/qmfx.h) with the reference's error
// convention: any failing call aborts through LOG(FATAL) with the library's message.
#pragma once

#include <cstdlib>
#include <string>

#include <qmfx.h>

#include <qmf/utils/Log.h>

namespace qmf {

// Which GPU and which arithmetic the engines use.  Defaults come from the environment
// (QMF_DEVICE, QMF_PRECISION), then device 0 and fp64 (the reference's `Double`,
// Types.h:24); the CLIs expose --device and --precision.  fp64 matches the reference's
// arithmetic to ~1e-12.  fp32 (opt-in) stores the factors in fp32: on well-posed problems it
// meets the 1e-4 factor tolerance at the reference's λ/α, but its error grows as cond·6e-8,
// so rank-deficient inputs (e.g. more factors than distinct fixed-side rows) need fp64.
//
// ngpus > 1 (--ngpus, QMF_NGPUS; WALS only) drives devices device .. device+ngpus-1 from this
// process: users and items are split into nnz-balanced row ranges, one per GPU, and every
// half-epoch ends with an RCCL all-gather of the solved rows (qmfx_dist_init_all,
// qmfx_wals_half_multi) — the reference's scheduler/labor bucket model
// (distributed/scheduler/RunOneTask.cpp:160-243) inside one node.
struct DeviceOptions {
  int device = envInt("QMF_DEVICE", 0);
  int precision = envInt("QMF_PRECISION", 64);
  int ngpus = envInt("QMF_NGPUS", 1);

  static int envInt(const char* name, int def) {
    const char* v = std::getenv(name);
    return v && *v ? std::atoi(v) : def;
  }
};

#define QMFX_CHECK(call)                                                              \
  do {                                                                                \
    const int qmfx_rc_ = (call);                                                      \
    if (qmfx_rc_ != 0)                                                                \
      LOG(FATAL) << #call << " failed (" << qmfx_rc_ << "): " << qmfx_last_error();   \
  } while (0)

class DeviceContext {
 public:
  DeviceContext(const DeviceOptions& opt, const size_t nfactors, const int deviceOffset = 0) {
    CHECK(opt.precision == 32 || opt.precision == 64)
      << "precision must be 32 or 64, got " << opt.precision;
    QMFX_CHECK(qmfx_create(&ctx_, opt.device + deviceOffset, opt.precision,
                           static_cast<int>(nfactors)));
  }
  ~DeviceContext() {
    if (ctx_) qmfx_destroy(ctx_);
  }
  DeviceContext(const DeviceContext&) = delete;
  DeviceContext& operator=(const DeviceContext&) = delete;

  qmfx_ctx* get() const { return ctx_; }

 private:
  qmfx_ctx* ctx_ = nullptr;
};

}  // namespace qmf

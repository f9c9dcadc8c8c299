// Minimal logging / CHECK facility for the drop-in host library.  Keeps the reference's
// conventions: LOG(INFO|WARNING|ERROR) to stderr, LOG(FATAL) and failed CHECKs abort the
// process (the reference uses glog, which is not part of this image).
#pragma once

#include <cstdlib>
#include <iostream>
#include <sstream>
#include <string>

namespace qmf {
namespace log {

enum Severity { INFO = 0, WARNING = 1, ERROR = 2, FATAL = 3 };

inline int& minLevel() {
  static int level = [] {
    const char* e = std::getenv("QMF_MINLOGLEVEL");
    return e ? std::atoi(e) : 0;
  }();
  return level;
}

class Message {
 public:
  Message(Severity s, const char* file, int line) : sev_(s) {
    static const char* tags = "IWEF";
    os_ << tags[s] << " " << file << ":" << line << "] ";
  }
  ~Message() {
    if (sev_ >= minLevel() || sev_ == FATAL) {
      os_ << '\n';
      std::cerr << os_.str();
      std::cerr.flush();
    }
    if (sev_ == FATAL) std::abort();
  }
  std::ostream& stream() { return os_; }

 private:
  Severity sev_;
  std::ostringstream os_;
};

struct Voidify {
  void operator&(std::ostream&) {}
};

}  // namespace log
}  // namespace qmf

#define QMF_LOG_INFO ::qmf::log::Message(::qmf::log::INFO, __FILE__, __LINE__).stream()
#define QMF_LOG_WARNING ::qmf::log::Message(::qmf::log::WARNING, __FILE__, __LINE__).stream()
#define QMF_LOG_ERROR ::qmf::log::Message(::qmf::log::ERROR, __FILE__, __LINE__).stream()
#define QMF_LOG_FATAL ::qmf::log::Message(::qmf::log::FATAL, __FILE__, __LINE__).stream()
#define LOG(sev) QMF_LOG_##sev

#define CHECK(cond) \
  (cond) ? (void)0 : ::qmf::log::Voidify() & QMF_LOG_FATAL << "Check failed: " #cond " "
#define QMF_CHECK_OP(a, b, op)                                                           \
  ((a)op(b)) ? (void)0                                                                   \
             : ::qmf::log::Voidify() & QMF_LOG_FATAL << "Check failed: " #a " " #op " " #b \
                                                     << " (" << (a) << " vs. " << (b) << ") "
#define CHECK_EQ(a, b) QMF_CHECK_OP(a, b, ==)
#define CHECK_NE(a, b) QMF_CHECK_OP(a, b, !=)
#define CHECK_GT(a, b) QMF_CHECK_OP(a, b, >)
#define CHECK_GE(a, b) QMF_CHECK_OP(a, b, >=)
#define CHECK_LT(a, b) QMF_CHECK_OP(a, b, <)
#define CHECK_LE(a, b) QMF_CHECK_OP(a, b, <=)

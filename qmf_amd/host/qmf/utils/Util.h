// String helpers (reference: qmf/utils/Util.h:24-27).
#pragma once

#include <string>
#include <vector>

namespace qmf {

// splits `str` on `delim`; an empty string gives no pieces, "a," gives {"a", ""}
std::vector<std::string> split(const std::string& str, const char delim);

}  // namespace qmf

// Base types of the drop-in host API (reference: qmf/Types.h:24).
#pragma once

#include <cstddef>
#include <cstdint>

namespace qmf {

// base type for floating point numbers on the host side of the API
using Double = double;

}  // namespace qmf

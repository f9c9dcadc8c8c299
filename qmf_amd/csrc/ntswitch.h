// Host-side dispatch of a runtime tile count to the kernel template instances.
#pragma once

#define QMFX_NT_SWITCH(NTV, CALL)         \
  switch (NTV) {                          \
    case 1: return CALL(1);               \
    case 2: return CALL(2);               \
    case 3: return CALL(3);               \
    case 4: return CALL(4);               \
    case 5: return CALL(5);               \
    case 6: return CALL(6);               \
    case 7: return CALL(7);               \
    case 8: return CALL(8);               \
    default: return hipErrorInvalidValue; \
  }
// fp32 whitened path: every one-wave tiling plus k = 256 (NT = 16, beside the multi-wave
// direct kernel)
#define QMFX_NT_SWITCH_W(NTV, CALL)       \
  switch (NTV) {                          \
    case 1: return CALL(1);               \
    case 2: return CALL(2);               \
    case 3: return CALL(3);               \
    case 4: return CALL(4);               \
    case 5: return CALL(5);               \
    case 6: return CALL(6);               \
    case 7: return CALL(7);               \
    case 8: return CALL(8);               \
    case 16: return CALL(16);             \
    default: return hipErrorInvalidValue; \
  }
#define QMFX_NT_SWITCH64(NTV, CALL)       \
  switch (NTV) {                          \
    case 1: return CALL(1);               \
    case 2: return CALL(2);               \
    case 3: return CALL(3);               \
    case 4: return CALL(4);               \
    default: return hipErrorInvalidValue; \
  }


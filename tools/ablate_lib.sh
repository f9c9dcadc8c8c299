#!/bin/bash
# Runs tools/ablate.py against alternative library builds (timing experiments).
for lib in "$@"; do echo "== $lib"; QMFX_LIB=$lib python tools/ablate.py; done

#!/bin/bash
# Build a wheel (native runtime compiled for gfx950 first). No upload: this
# environment has no package index access; publish the dist/ artefacts manually.
set -euo pipefail
cd "$(dirname "$0")"
python -c "from elephas_amd import _build; print(_build.build(verbose=True))"
python -m pip wheel --no-deps --no-build-isolation -w dist .

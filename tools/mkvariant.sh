#!/bin/bash
# Build an A/B variant of the library with extra HIP flags into ab_libs/NAME.so,
# then restore the default build.  usage: bash tools/mkvariant.sh NAME -DFLAG ...
set -e
cd "$(dirname "$0")/.."
name=$1; shift
mkdir -p ab_libs
python -c "import sys; sys.path.insert(0, 'isaklm-raytracer_amd'); import build; build.build(extra_hip_flags=sys.argv[1:])" "$@"
cp isaklm-raytracer_amd/libisaklm_rt.so ab_libs/$name.so
python -c "import sys; sys.path.insert(0, 'isaklm-raytracer_amd'); import build; build.build()"
echo "ab_libs/$name.so"

#!/bin/bash
# Build the standalone timing probes into probe_build/ (git-ignored; travels to the GPU box).
set -e
cd "$(dirname "$0")/../.."
mkdir -p probe_build
for f in tools/probe/*.hip; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 "$f" -o probe_build/$(basename "$f" .hip)
done

#!/bin/bash
# builds tools/microbench/bin/torch_host_cost (see torch_host_cost.cc)
set -e
cd "$(dirname "$0")"
mkdir -p bin
eval "$(python - <<'EOF'
import torch
from torch.utils import cpp_extension as ce
print('TINC="%s"' % " ".join("-isystem " + p for p in ce.include_paths()))
print('TLIB="%s"' % ce.library_paths()[0])
print('ABI=%d' % int(torch._C._GLIBCXX_USE_CXX11_ABI))
EOF
)"
g++ -O2 -std=c++17 -D_GLIBCXX_USE_CXX11_ABI=$ABI -D__HIP_PLATFORM_AMD__ -DUSE_ROCM \
  -isystem /opt/rocm/include $TINC torch_host_cost.cc -o bin/torch_host_cost \
  -Wl,--no-as-needed -L$TLIB -Wl,-rpath,$TLIB -lc10 -lc10_hip -ltorch -ltorch_cpu -ltorch_hip \
  -L/opt/rocm/lib -Wl,-rpath,/opt/rocm/lib -lamdhip64

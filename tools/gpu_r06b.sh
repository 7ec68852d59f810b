set -o pipefail
tools/gpu_ab_lazy62.sh && tools/gpu_tensor_traffic.sh

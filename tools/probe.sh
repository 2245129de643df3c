set -x
python -c "import torch; print('torch only', torch.cuda.is_available(), torch.cuda.device_count()); x=torch.ones(3,device='cuda'); print(x.sum())" 2>&1 | tail -3
python -c "
import sys; sys.path.insert(0,'jieba-go_amd/python')
import ctypes, jiebahip as J
L=ctypes.CDLL('libamdhip64.so'); n=ctypes.c_int(); print('hipGetDeviceCount', L.hipGetDeviceCount(ctypes.byref(n)), n.value)
import torch; print('after hip', torch.cuda.is_available(), torch.cuda.device_count())
" 2>&1 | tail -3
env | grep -i -E "hip|rocr|cuda|gpu" | head
ls /opt/rocm/lib/libamdhip64* ; python -c "import torch; print(torch.version.hip)"

import sys, os
sys.path[:0] = ['vvc-extension-mm_amd', '.']
import mm360
mm360.LIB_PATH = os.path.abspath('tmp_variants/dbgdiv/libmm360.so')
from mm360 import workload as W
for name in ('C1', 'C2', 'C3'):
    cfg = W.CONFIGS[name]
    with mm360.MMContext(mm360.seq_params(cfg.width, cfg.height, cfg.models), device=0) as ctx:
        pass

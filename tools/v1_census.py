"""Strict full-message census of the reference v1 configs (tests/test_v1_configs_all_cpu.py): exact count and the first diffs of each config."""
import sys, os, glob
sys.path.insert(0, "tests"); sys.path.insert(0, ".")
import test_v1_configs_all_cpu as T
import paddle_amd.trainer_config_helpers as tch
from paddle_amd.trainer_config_helpers import config_proto as cp
ex=[]; bad={}
only = sys.argv[1:]
for f in sorted(glob.glob(os.path.join(T.REF,"*.py"))):
    n=os.path.basename(f)[:-3]
    if only and n not in only: continue
    pp=os.path.join(T.REF,"protostr",n+".protostr")
    if not os.path.exists(pp): continue
    txt = open(pp).read()
    whole = txt.lstrip().startswith("model_config")
    exp=cp.from_text("TrainerConfig" if whole else "ModelConfig", txt, strict=True)
    try:
        c = tch.parse_config(f)
        got = c.trainer_config() if whole else c.model_config()
        d=T._diff(got,exp)
        if not d: ex.append(n)
        else: bad[n]=(len(d), d[:6])
    except Exception as e: bad[n]=("ERR", repr(e)[:150])
print("strict exact:", len(ex))
for k,v in bad.items(): print(k, v)

# variant: software-pipelined attention (tools/variants/attention_pp.hip replaces attention.hip)
import shutil
import sys
from pathlib import Path
shutil.copy(Path(__file__).with_name("attention_pp.hip"), sys.argv[1] + "/attention.hip")

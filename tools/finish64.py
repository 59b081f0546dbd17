"""The finish phase (extract_skeleton + extract_faces) on the synth64h
complex, for profiling: python tools/finish64.py (prints bench.finish_check)."""
import json
import os
import sys

sys.path[:0] = [os.getcwd(), os.path.join(os.getcwd(), "tropical-nerf.pytorch_amd"), os.path.join(os.getcwd(), "tests")]
import torch  # noqa: E402

from bench import finish_check  # noqa: E402

print(json.dumps(finish_check(torch.device("cuda", 0), reps=3)))

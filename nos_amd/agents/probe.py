"""Per-slice throughput probe of the CU-mask gpuagent (SURVEY.md 2.1 [NEW]).

For a GPU whose slice table has ``n`` slices, the device plugin's ``even``
CU policy gives each slice ``32 // n`` CUs per XCD; the probe runs the gfx950
MFMA-peak and HBM-stream kernels (``csrc/hip/probes.hip``) on a stream
restricted to the first such slice and reports TFLOP/s and GB/s, which the
reporter publishes as node annotations (``nos.nebuly.com/probe-gpu-<i>-<profile>-tflops|gbps``)
so schedulers/operators can see what a slice really delivers.
"""
from __future__ import annotations

import logging

from ..gpu.topology import MI355X_CUS_PER_XCD, split_even

log = logging.getLogger("nos_amd.agents.probe")


class SliceProber:
    def __init__(self, smi, plugin=None, iters: int = 4000):
        self.smi = smi
        self.plugin = plugin
        self.iters = iters

    def _slices_on(self, gpu: int) -> int:
        if self.plugin is None:
            return 1
        return max(1, sum(1 for d in self.plugin.devices.values()
                          if d.gpu_index == gpu and d.resource.startswith("amd.com/gpu-")))

    def __call__(self, gpu: int, profile: str) -> dict:
        import torch

        from ..ops import probes
        from ..ops.streams import CUMaskedStream, device_info

        n = min(self._slices_on(gpu), MI355X_CUS_PER_XCD)
        info = device_info(gpu)
        cus = split_even(n)[0].cus()
        s = CUMaskedStream(cus, info["num_cus"], device=gpu)
        try:
            with torch.cuda.device(gpu):
                tf = probes.mfma_peak_tflops(s.handle, nwg=len(cus) * 4, iters=self.iters)
                gbps = probes.hbm_gbps(s.handle, bytes_=256 << 20, iters=3, nwg=len(cus) * 4)
        finally:
            s.close()
        log.info("gpu %d slice %s (%d CUs): %.1f TFLOP/s, %.0f GB/s", gpu, profile, len(cus), tf, gbps)
        return {"tflops": tf, "gbps": gbps, "cus": len(cus)}

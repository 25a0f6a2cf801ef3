"""Per-slice throughput probe of the CU-mask gpuagent (SURVEY.md 2.1 [NEW]).

For every (GPU, slice profile) the probe runs the gfx950 probe kernels
(``csrc/hip/probes.hip``) on a stream restricted to exactly the CUs the device
plugin gives a slice of that profile (its XCD-symmetric slot set), and reports:

* ``tflops``      -- register-only MFMA peak of those CUs (the chip's clock ceiling);
* ``gemmtflops``  -- the LDS-tiled bf16 MFMA GEMM (gemm.hip, 4096^3, one
  tile per workgroup, dispatched only to the slice CUs): what a tenant's matmuls get;
* ``gbps``        -- HBM read stream (8 x 16 B per lane in flight, 32
  workgroups per CU, non-temporal: 6.4 TB/s on the whole MI355X);
* ``sclkmhz``     -- the GFX clock amd-smi reads right after the MFMA probe
  (separates DVFS from a kernel limit);
* ``loadedgbps`` / ``loadedgemmtflops`` -- the same while a synthetic
  co-tenant load (HBM copies + MFMA) runs on the complement CUs: what the
  slice delivers when its neighbours are busy.

The reporter publishes them as node annotations
``nos.nebuly.com/probe-gpu-<i>-<profile>-<metric>``; the partitioner scores
slices on ``gemmtflops`` when present (:mod:`nos_amd.partitioning.scoring`).
"""
from __future__ import annotations

import logging

from ..gpu.topology import MI355X_CUS_PER_XCD, MI355X_MEMORY_GB, MI355X_XCDS, logical_cu, slot_wants

log = logging.getLogger("nos_amd.agents.probe")

METRICS = ("tflops", "gemmtflops", "gbps", "sclkmhz", "loadedgbps", "loadedgemmtflops")


def _profile_gb(profile: str) -> int:
    return int(profile[:-2]) if profile.endswith("gb") and profile[:-2].isdigit() else 0


class SliceProber:
    def __init__(self, smi, plugin=None, iters: int = 4000, loaded: bool = True, gemm_n: int = 4096):
        self.smi = smi
        self.plugin = plugin
        self.iters = iters
        self.loaded = loaded
        self.gemm_n = gemm_n

    def slice_cus(self, gpu: int, profile: str, num_cus: int) -> list[int]:
        """The CU set a slice of ``profile`` on ``gpu`` runs on: a live replica's
        slots from the device plugin, else the proportional share."""
        if self.plugin is not None:
            for d in sorted(self.plugin.devices.values(), key=lambda d: d.id):
                if d.gpu_index == gpu and d.profile == profile and self.plugin.cus_of(d.id):
                    return self.plugin.cus_of(d.id)
        per_xcd = slot_wants([("x", _profile_gb(profile) or MI355X_MEMORY_GB)], "proportional",
                             MI355X_MEMORY_GB)["x"]
        xcds = MI355X_XCDS if num_cus >= MI355X_XCDS else 1
        return sorted(logical_cu(x, j, xcds) for x in range(xcds) for j in range(min(per_xcd, MI355X_CUS_PER_XCD)))

    def __call__(self, gpu: int, profile: str) -> dict:
        import torch

        from ..ops import probes
        from ..ops.streams import CUMaskedStream, device_info

        info = device_info(gpu)
        cus = self.slice_cus(gpu, profile, info["num_cus"])
        comp = sorted(set(range(info["num_cus"])) - set(cus))
        s = CUMaskedStream(cus, info["num_cus"], device=gpu)
        out: dict = {"cus": len(cus)}
        try:
            with torch.cuda.device(gpu):
                out["tflops"] = probes.mfma_peak_tflops(s.handle, nwg=len(cus) * 4, iters=self.iters)
                try:
                    out["sclkmhz"] = float(self.smi.clock(gpu)["sclk_mhz"])
                except Exception:  # clock unreadable on this backend: omit it
                    pass
                out["gemmtflops"] = probes.gemm_tflops(s.handle, n=self.gemm_n, iters=3)
                out["gbps"] = probes.hbm_mode_gbps(s.handle, "read", 512 << 20, 3, nwg=32 * len(cus))
                if self.loaded and comp:
                    out.update(self._loaded(s, comp, info["num_cus"], gpu))
        finally:
            s.close()
        log.info("gpu %d slice %s (%d CUs): %s", gpu, profile, len(cus),
                 {k: round(v, 1) for k, v in out.items() if isinstance(v, float)})
        return out

    def _loaded(self, s, comp: list[int], num_cus: int, gpu: int) -> dict:
        """Re-measure the slice while HBM copies and MFMA chains keep the other CUs busy."""
        import torch

        from ..ops import _lib, probes
        from ..ops.streams import CUMaskedStream

        bg = CUMaskedStream(comp, num_cus, device=gpu)
        try:
            a = torch.empty(256 << 20, dtype=torch.uint8, device=f"cuda:{gpu}")
            b = torch.empty_like(a)
            scratch = torch.empty(len(comp) * 4, dtype=torch.float32, device=f"cuda:{gpu}")
            with torch.cuda.stream(bg.torch):
                for _ in range(40):  # ~ seconds of co-tenant traffic, enqueued up front
                    b.copy_(a)
                    _lib.check(_lib.lib().nos_probe_mfma_peak_launch(bg.handle, len(comp) * 2, 2000,
                                                                     scratch.data_ptr()), "mfma_load")
            out = {"loadedgbps": probes.hbm_mode_gbps(s.handle, "read", 512 << 20, 3, nwg=32 * len(s.cus)),
                   "loadedgemmtflops": probes.gemm_tflops(s.handle, n=self.gemm_n, iters=3)}
            bg.synchronize()
            return out
        finally:
            bg.close()

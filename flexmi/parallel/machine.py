"""MI355X machine model for the execution simulator.

Reference: the simulator's machine is a set of GPUs with pairwise intra-node links
(20·2^20 B/ms ≈ 21 GB/s), inter-node links (12·2^20/numNodes B/ms) and GPU<->DRAM links
(``src/runtime/simulator.cu:21-76``), sized for the NVLink/PCIe era.

flexmi models one MI355X node as 8 GPUs on a full xGMI mesh (7 links per GPU, ≈153 GB/s
per link), 288 GB HBM3E per GPU (≈6.3 TB/s measured stream bandwidth, guides/MI355X_MICROARCH.md),
PCIe Gen5 x16 to the host (63 GB/s), and RCCL collectives (ring all-reduce cost
``lat + 2(g-1)/g · bytes / busbw``).  Link and collective constants are spec-derived and
*uncalibrated* above one GPU (the 1-GPU box cannot measure xGMI); they can be overridden with a
JSON file (``--machine``) once measured on an 8-GPU node.
"""
from __future__ import annotations

import json
from dataclasses import asdict, dataclass


@dataclass
class MachineModel:
    ndev: int = 8
    gpus_per_node: int = 8
    # effective per-direction point-to-point bandwidth between two GPUs of a node (one xGMI
    # link, RCCL send/recv efficiency ~0.6 of the 153 GB/s link rate for mid-size messages)
    link_GBps: float = 90.0
    link_lat_us: float = 8.0
    nic_GBps: float = 45.0
    nic_lat_us: float = 15.0
    # RCCL ring all-reduce bus bandwidth with all 8 GPUs of a node (uses every link)
    ar_busbw_GBps: float = 320.0
    ar_lat_us: float = 20.0
    hbm_bytes: float = 288e9 * 0.92
    hbm_GBps: float = 6300.0
    host_GBps: float = 63.0
    # compute roofline
    peak_bf16_tflops: float = 2500.0
    peak_fp32_tflops: float = 157.3
    mfma_eff: float = 0.22          # achieved/peak on DLRM-sized GEMMs (profiles/: 240-560 TF)
    hbm_eff: float = 0.75
    launch_us: float = 1.6          # kernel boundary inside a hipGraph replay
    # shortest launch inside a replayed step: small-batch layers are launch-bound, not roofline-bound.
    # 4.0 puts the 1-GPU projections of run_random / criteo_kaggle (batch 256) at +5 % / -20 % of
    # the measured steps, from -13 % / -57 % without it (tools/soap_report.py, profiles/soap_vs_dp_fp32.txt)
    kernel_floor_us: float = 4.0
    atomic_TBps: float = 1.3        # chip-wide fp32 atomic add rate (MI355X_MICROARCH.md)
    bucket_mb: float = 32.0
    overlap: bool = True
    # micro-batch pipelining of the exchange into the sample-split tail (executor
    # FLEXMI_XCHG_CHUNKS); 0 = the executor's auto rule for the model's per-GPU batch
    xchg_chunks: int = 0
    chunk_us: float = 1.6           # extra kernel boundaries per chunk and op

    @staticmethod
    def mi355x(ndev=8, **kw):
        m = MachineModel(ndev=ndev)
        for k, v in kw.items():
            setattr(m, k, v)
        return m

    @staticmethod
    def load(path, ndev=None):
        with open(path) as f:
            d = json.load(f)
        m = MachineModel(**{k: v for k, v in d.items() if k in MachineModel.__dataclass_fields__})
        if ndev is not None:
            m.ndev = ndev
        return m

    def save(self, path):
        with open(path, "w") as f:
            json.dump(asdict(self), f, indent=1)

    def native_dict(self):
        return {"ndev": self.ndev, "gpus_per_node": self.gpus_per_node, "link_GBps": self.link_GBps,
                "link_lat_us": self.link_lat_us, "nic_GBps": self.nic_GBps, "nic_lat_us": self.nic_lat_us,
                "ar_busbw_GBps": self.ar_busbw_GBps, "ar_lat_us": self.ar_lat_us, "hbm_bytes": self.hbm_bytes,
                "bucket_bytes": self.bucket_mb * (1 << 20), "overlap": self.overlap,
                "xchg_chunks": int(self.xchg_chunks), "chunk_us": self.chunk_us}

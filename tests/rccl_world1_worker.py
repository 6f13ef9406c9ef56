"""Worker for tests/test_gpu_rccl.py: a ONE-rank ``nccl`` (RCCL) process group on cuda:0,
initialised exactly as flexmi.parallel.comm.init_distributed does for a multi-GPU run (device_id
bound), then every collective kind of the native step runner (flexmi._rt) -- all-to-all, grouped
point-to-point (start/endCoalescing), all-reduce (async + sync), reduce-scatter, all-gather --
plus the executor-level fused exchange and sparse-DP all-gather items, checked against torch.
Prints "rccl world1 ok" on success; any mismatch raises."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    os.environ.update(RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1")
    os.environ.setdefault("MASTER_PORT", sys.argv[1] if len(sys.argv) > 1 else "29512")
    import torch
    import torch.distributed as dist
    from flexmi.parallel.comm import Comm
    import datetime
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", timeout=datetime.timedelta(seconds=60), device_id=torch.device("cuda", 0))
    comm = Comm()
    assert dist.get_backend() == "nccl" and comm.backend == "nccl" and comm.world == 1
    from flexmi import _rt
    dev = torch.device("cuda")
    pg = dist.group.WORLD
    rt = _rt.StepRunner()
    pid = rt.new_program()
    s = [rt.new_slot() for _ in range(8)]
    torch.manual_seed(0)
    a2a_send = torch.randn(4096, device=dev)
    a2a_recv = torch.empty_like(a2a_send)
    rt.add_all_to_all(pid, s[0], pg, a2a_recv, a2a_send, [4096], [4096], "a2a")
    rt.add_wait(pid, s[0], "a2a.wait")
    p2p_send = torch.randn(1000, device=dev)
    p2p_recv = torch.zeros_like(p2p_send)
    rt.add_p2p(pid, s[1], pg, p2p_recv, p2p_send, [1000], [1000], "p2p")
    rt.add_wait(pid, s[1], "p2p.wait")
    ar = torch.randn(3001, device=dev)
    ar_ref = ar.clone()
    rt.add_all_reduce(pid, s[2], pg, ar, False, "ar.start")
    rt.add_wait(pid, s[2], "ar.wait")
    ar2 = torch.randn(777, device=dev)
    ar2_ref = ar2.clone()
    rt.add_all_reduce(pid, s[3], pg, ar2, True, "ar.sync")
    rs_in = torch.randn(2048, device=dev)
    rs_out = torch.zeros(2048, device=dev)
    rt.add_reduce_scatter(pid, s[4], pg, rs_out, rs_in, True, "rs")
    ag_in = torch.randn(640, device=dev)
    ag_out = torch.zeros(640, device=dev)
    rt.add_all_gather(pid, s[5], pg, ag_out, ag_in, "ag")
    bf = torch.randn(512, device=dev).to(torch.bfloat16)
    bf_out = torch.zeros_like(bf)
    rt.add_all_to_all(pid, s[6], pg, bf_out, bf, [512], [512], "a2a.bf16")
    rt.add_wait(pid, s[6], "a2a.bf16.wait")
    for _ in range(3):                      # repeated runs reuse the slots
        rt.run(pid)
    torch.cuda.synchronize()
    assert torch.equal(a2a_recv, a2a_send), "all_to_all"
    assert torch.equal(p2p_recv, p2p_send), "grouped p2p"
    assert torch.equal(ar, ar_ref) and torch.equal(ar2, ar2_ref), "all_reduce (world 1 = identity)"
    assert torch.equal(rs_out, rs_in), "reduce_scatter"
    assert torch.equal(ag_out, ag_in), "all_gather"
    assert torch.equal(bf_out, bf), "bf16 all_to_all"
    st = rt.stats()
    assert st["collectives"] == 3 * 7 and st["runs"] == 3, st
    # the Python Comm layer over the same RCCL communicator
    x = torch.randn(100, device=dev)
    out = comm.all_to_all([x], [100], torch.float32, dev)
    assert torch.equal(out[0], x)
    y = torch.randn(64, device=dev)
    y0 = y.clone()
    comm.all_reduce_op(y, op="max")
    assert torch.equal(y, y0)
    # a subset communicator of the single rank (what the plan compiler creates for replica sets)
    g = dist.new_group([0])
    z = torch.randn(32, device=dev)
    z0 = z.clone()
    dist.all_reduce(z, group=g)
    torch.cuda.synchronize()
    assert torch.equal(z, z0)
    rt.release()
    dist.barrier()
    dist.destroy_process_group()
    print("rccl world1 ok", flush=True)


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""The early-step phase of the bench: per-step kernel times
beside the GPU's clocks and power, from evidence instead of by hypothesis.

Runs bench.py's workload (RotatE FB15k shape, b=1024, n=256, fused Adam) for
--steps steps back to back with no host wait, the stage timer on every step
(kge_stage_timer command 3: each step's k_row and entity-pass time and its
start on the device clock), while a host thread samples amdsmi — current GFX
and memory clocks, socket power, hotspot / HBM temperature, and the GFX
activity — every ~0.25 ms.  The two series are aligned on the device clock
through one synchronised start; the output lists both per step.

    python tools/hump_trace.py --bursts 0:150,1000:60,50:60,5000:60 > gpurun_out/hump.jsonl

Bursts "idle_ms:steps": after the first burst, the GPU idles idle_ms before
the next one — whether the early-step phase returns after an idle gap in the
same process, and after how long, separates a power-state effect from one of
the process's own data.

--clock-probe: the SMU's metrics table refreshes every ≈20 ms, too coarse for
a phase of ≈10 steps (≈6 ms), so the shader clock is also read in-kernel:
tools/dbg/libclock_probe.so's one-wave kernel runs on a second stream through
each burst and samples (s_memrealtime, s_memtime) every few µs; each step's
row-pass and entity-pass clock is Δtick / Δreal × 100 MHz over the samples
inside that kernel's event-timed interval (placed on the probe's time axis by
a marker kernel on the step stream just before the burst).
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import threading
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

import bench  # noqa: E402
from knowledgegraphembedding_amd import KGEAdam, KGEModel, _lib  # noqa: E402


def sampler(handle, out, stop):
    """amdsmi's GPU metrics table (the SMU's own values; it refreshes every
    few ms — firmware_timestamp tells when): per-XCC GFX clocks, SOC clocks,
    the memory clock, the energy accumulator (power over any interval), the
    throttle flags and residency counters."""
    import amdsmi as A
    while not stop.is_set():
        t = time.perf_counter()
        rec = {"t": t}
        try:
            m = A.amdsmi_get_gpu_metrics_info(handle)
            for k in ("firmware_timestamp", "energy_accumulator", "current_uclk", "throttle_status",
                      "ppt_residency_acc", "prochot_residency_acc", "socket_thm_residency_acc", "hbm_thm_residency_acc",
                      "current_socket_power", "average_gfx_activity", "average_umc_activity", "temperature_hotspot",
                      "temperature_mem"):
                v = m.get(k)
                if isinstance(v, (int, float, bool)):
                    rec[k] = float(v)
            for k in ("current_gfxclks", "current_socclks"):
                v = [x for x in (m.get(k) or []) if isinstance(x, (int, float)) and 0 < x < 10000]
                if v:
                    rec[k] = float(np.mean(v))
        except Exception as e:  # noqa: BLE001
            rec["err"] = str(e)[:80]
        out.append(rec)
        time.sleep(0.0002)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bursts", default="0:150,1000:60,50:60,5000:60")
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--clock-probe", default=os.path.join(HERE, "dbg", "libclock_probe.so"),
                    help="in-kernel clock probe library ('' = off)")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    import amdsmi as A
    A.amdsmi_init()
    handles = A.amdsmi_get_processor_handles()
    handle = handles[0]
    # the amdsmi handle of the device torch uses (amdsmi lists every GPU of the host)
    props = torch.cuda.get_device_properties(dev)
    bus = getattr(props, "pci_bus_id", None)
    for h in handles:
        try:
            bdf = A.amdsmi_get_gpu_device_bdf(h)  # "0000:bb:dd.f"
            if bus is not None and int(bdf.split(":")[1], 16) == int(bus):
                handle = h
        except Exception:  # noqa: BLE001
            pass
    print(json.dumps({"gpus_seen_by_amdsmi": len(handles), "torch_pci_bus": bus,
                      "bdf": A.amdsmi_get_gpu_device_bdf(handle)}))
    torch.manual_seed(0)
    model = KGEModel("RotatE", bench.E, bench.R, bench.D, bench.GAMMA, True, False).to(dev)
    opt = KGEAdam([p for p in model.parameters() if p.requires_grad], lr=1e-4)
    from argparse import Namespace
    args = Namespace(cuda=True, negative_adversarial_sampling=True, adversarial_temperature=1.0, uni_weight=False,
                     regularization=0.0, dp_group=None)
    it = bench.DeviceBatches(dev, seed=1000)
    for _ in range(a.warmup):
        KGEModel.train_step(model, opt, it, args)
    torch.cuda.synchronize()
    lib = _lib.load()
    probe = None
    if a.clock_probe and os.path.exists(a.clock_probe):
        probe = ctypes.CDLL(a.clock_probe)
        probe.clock_probe_launch.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
        probe.marker_stamp.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        probe_stream = torch.cuda.Stream(dev)
    samples, stop = [], threading.Event()
    th = threading.Thread(target=sampler, args=(handle, samples, stop), daemon=True)
    th.start()
    time.sleep(0.05)
    keys = ("current_gfxclks", "current_socclks", "current_uclk", "current_socket_power", "throttle_status",
            "average_gfx_activity", "average_umc_activity", "temperature_hotspot", "temperature_mem")
    # bursts "idle_ms:steps,...": the GPU idles idle_ms before each burst of back-to-back steps
    for bi, spec in enumerate(a.bursts.split(",")):
        idle_ms, nsteps = (float(x) for x in spec.split(":"))
        nsteps = int(nsteps)
        time.sleep(idle_ms / 1e3)
        if probe is not None:
            nsamp = int((nsteps * 0.7 + 10.0) / 0.0035)  # ≈3.5 µs per sample (one s_sleep 127)
            pbuf = torch.zeros(2 * nsamp, dtype=torch.int64, device=dev)
            mbuf = torch.zeros(2, dtype=torch.int64, device=dev)
            torch.cuda.synchronize()
            assert probe.clock_probe_launch(pbuf.data_ptr(), nsamp, 1, ctypes.c_void_p(probe_stream.cuda_stream)) == 0
            assert probe.marker_stamp(mbuf.data_ptr(), ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)) == 0
        _lib.check(lib.kge_stage_timer(1, None, 1), "kge_stage_timer")
        t_host0 = time.perf_counter()
        for _ in range(nsteps):
            KGEModel.train_step(model, opt, it, args)
        torch.cuda.synchronize()
        t_host1 = time.perf_counter()
        buf = np.zeros(7 * nsteps, dtype=np.float32)
        _lib.check(lib.kge_stage_timer(3, buf.ctypes.data_as(ctypes.c_void_p), buf.size), "kge_stage_timer")
        lib.kge_stage_timer(0, None, 0)
        st = buf.reshape(nsteps, 7)
        clk = None
        if probe is not None:
            torch.cuda.synchronize()
            pv = pbuf.cpu().numpy().reshape(-1, 2).astype(np.float64)
            mv = mbuf.cpu().numpy().astype(np.float64)
            pv = pv[pv[:, 0] > 0]
            t_ms = (pv[:, 0] - mv[0]) / 1e5  # 100 MHz constant counter → ms from the marker

            def clock_mhz(t0, t1):
                sel = np.nonzero((t_ms >= t0) & (t_ms <= t1))[0]
                if len(sel) < 2:
                    return None
                i, j = sel[0], sel[-1]
                return float((pv[j, 1] - pv[i, 1]) / (pv[j, 0] - pv[i, 0]) * 100.0)
            clk = clock_mhz
        print(json.dumps({"burst": bi, "idle_ms_before": idle_ms, "steps": nsteps,
                          "host_span_ms": (t_host1 - t_host0) * 1e3,
                          "device_span_ms": float(st[-1, 6] + st[-1, :6].sum())}), flush=True)
        snap = list(samples)
        for k in range(nsteps):
            t0 = t_host0 + st[k, 6] / 1e3
            t1 = t0 + st[k, :6].sum() / 1e3
            win = [s_ for s_ in snap if t0 - 0.0005 <= s_["t"] <= t1 + 0.0005]
            agg = {}
            for key in keys:
                v = [s_[key] for s_ in win if key in s_]
                if v:
                    agg[key] = float(np.mean(v))
            fts = sorted({s_["firmware_timestamp"] for s_ in win if "firmware_timestamp" in s_})
            rec = {"burst": bi, "step": k, "row_ms": float(st[k, 1]), "entity_ms": float(st[k, 4]),
                   "start_ms": float(st[k, 6]), "n_samples": len(win), "fw_stamps": len(fts), **agg}
            if clk is not None:
                s0 = float(st[k, 6])
                rec["probe_row_mhz"] = clk(s0 + float(st[k, 0]), s0 + float(st[k, :2].sum()))
                rec["probe_entity_mhz"] = clk(s0 + float(st[k, :4].sum()), s0 + float(st[k, :5].sum()))
            print(json.dumps(rec))
    time.sleep(0.05)
    stop.set()
    th.join()
    # the metrics table's own refresh: distinct firmware timestamps per second of sampling
    fts = [s_["firmware_timestamp"] for s_ in samples if "firmware_timestamp" in s_]
    span = samples[-1]["t"] - samples[0]["t"] if samples else 0.0
    print(json.dumps({"samples": len(samples), "distinct_fw_stamps": len(set(fts)), "span_s": span,
                      "energy_first_last": [samples[0].get("energy_accumulator"), samples[-1].get("energy_accumulator")]
                      if samples else None}))
    A.amdsmi_shut_down()


if __name__ == "__main__":
    main()

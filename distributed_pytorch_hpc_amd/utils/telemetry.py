"""GPU clock / power / temperature telemetry for benchmark runs (amdsmi, host side only).

A background thread samples the rank's own MI355X through amdsmi's gpu-metrics table (one SMU table read per
sample: per-XCD current GFX clocks, socket power, hotspot / HBM temperature, throttle-residency accumulators) every
``period`` seconds.  Nothing here touches a HIP stream or synchronises the device, so the sampler can run across a
timed region.  Energy comes from the SMU energy accumulator read at the region's two edges (``mark()``), so it is
the integral over exactly the timed steps, not an estimate from sampled power.

Why it exists: the 7B step's GEMMs and attention are MFMA-dense, and MI355X lowers its clock under such load
(DVFS); the same binary then runs a few percent apart on different boxes.  A bench line that carries the clock it
held, the power it drew and the fraction of time the power limit (PPT) was active tells a kernel regression from
a slow box.  Reference counterpart: the per-rank GPU property report of tests/check_environment.py:118-179.

    tel = GpuTelemetry(device_index)      # starts sampling
    tel.mark("timed_start"); ...; tel.mark("timed_end")
    rec.update(tel.summary("timed_start", "timed_end"))
"""
from __future__ import annotations

import os
import threading
import time
from typing import Any, Dict, List, Optional

_NA16 = 0xFFFF


def _valid(v) -> bool:
    return isinstance(v, (int, float)) and 0 < v < _NA16


def _pct(vals: List[float], f: float) -> float:
    s = sorted(vals)
    return s[min(len(s) - 1, max(0, round(f * (len(s) - 1))))]


def _spread(vals: List[float], nd: int = 1) -> Optional[Dict[str, float]]:
    if not vals:
        return None
    return {"median": round(_pct(vals, 0.5), nd), "p10": round(_pct(vals, 0.1), nd),
            "p90": round(_pct(vals, 0.9), nd), "min": round(min(vals), nd), "max": round(max(vals), nd),
            "n": len(vals)}


def _bdf_of_torch_device(index: int) -> Optional[str]:
    try:
        import torch

        pr = torch.cuda.get_device_properties(index)
        dom = getattr(pr, "pci_domain_id", 0)
        bus = getattr(pr, "pci_bus_id", None)
        devid = getattr(pr, "pci_device_id", None)
        if bus is None or devid is None:
            return None
        return f"{dom:04x}:{bus:02x}:{devid:02x}"
    except Exception:   # noqa: BLE001 -- telemetry never fails a run
        return None


class GpuTelemetry:
    """Sample one GPU's clocks / power / temperatures on a host thread (see module docstring)."""

    def __init__(self, device_index: int = 0, period: float = 0.1, start: bool = True):
        self.period = period
        self.samples: List[Dict[str, Any]] = []
        self.marks: Dict[str, Dict[str, Any]] = {}
        self.error: Optional[str] = None
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None
        self._smi = None
        self._h = None
        try:
            import amdsmi

            amdsmi.amdsmi_init()
            self._smi = amdsmi
            handles = amdsmi.amdsmi_get_processor_handles()
            want = _bdf_of_torch_device(device_index)
            self._h = None
            if want:
                for h in handles:
                    try:
                        bdf = amdsmi.amdsmi_get_gpu_device_bdf(h).lower()
                    except Exception:   # noqa: BLE001
                        continue
                    if bdf.startswith(want):
                        self._h = h
                        break
            if self._h is None:
                # visible-device remapping without a BDF match: the n-th visible GPU
                vis = os.environ.get("HIP_VISIBLE_DEVICES") or os.environ.get("ROCR_VISIBLE_DEVICES") or \
                    os.environ.get("CUDA_VISIBLE_DEVICES")
                idx = device_index
                if vis:
                    try:
                        idx = int(vis.split(",")[device_index])
                    except (ValueError, IndexError):
                        pass
                self._h = handles[idx] if idx < len(handles) else (handles[0] if handles else None)
            if self._h is None:
                raise RuntimeError("amdsmi sees no GPU")
        except Exception as e:   # noqa: BLE001 -- no amdsmi / no GPU: the bench runs without telemetry
            self.error = f"{type(e).__name__}: {e}"
            self._smi = None
        if start and self._smi is not None:
            self._thread = threading.Thread(target=self._run, name="dph-telemetry", daemon=True)
            self._thread.start()

    # ---------------------------------------------------------------------------------------------------------
    def _read(self) -> Optional[Dict[str, Any]]:
        smi, h = self._smi, self._h
        try:
            m = smi.amdsmi_get_gpu_metrics_info(h)
        except Exception as e:   # noqa: BLE001
            self.error = f"metrics: {e}"
            return None
        clks = m.get("current_gfxclks")
        if isinstance(clks, (list, tuple)):
            clks = [c for c in clks if _valid(c)]
        else:
            clks = []
        sclk = sum(clks) / len(clks) if clks else (m.get("current_gfxclk") if _valid(m.get("current_gfxclk")) else None)
        pw = m.get("current_socket_power")
        if not _valid(pw):
            pw = m.get("average_socket_power") if _valid(m.get("average_socket_power")) else None
        return {"t": time.perf_counter(), "sclk": sclk, "sclk_min_xcd": min(clks) if clks else None, "power": pw,
                "temp_hot": m.get("temperature_hotspot") if _valid(m.get("temperature_hotspot")) else None,
                "temp_mem": m.get("temperature_mem") if _valid(m.get("temperature_mem")) else None}

    def _accumulators(self) -> Dict[str, Any]:
        smi, h = self._smi, self._h
        out: Dict[str, Any] = {"t": time.perf_counter()}
        try:
            e = smi.amdsmi_get_energy_count(h)
            out["energy_j"] = e["energy_accumulator"] * e["counter_resolution"] * 1e-6
        except Exception:   # noqa: BLE001
            pass
        try:
            m = smi.amdsmi_get_gpu_metrics_info(h)
            for k in ("accumulation_counter", "ppt_residency_acc", "socket_thm_residency_acc",
                      "prochot_residency_acc", "hbm_thm_residency_acc"):
                v = m.get(k)
                if isinstance(v, int):
                    out[k] = v
        except Exception:   # noqa: BLE001
            pass
        return out

    def _run(self):
        while not self._stop.is_set():
            s = self._read()
            if s is not None:
                self.samples.append(s)
            self._stop.wait(self.period)

    # ---------------------------------------------------------------------------------------------------------
    def mark(self, name: str) -> None:
        """Record the energy / throttle accumulators and the time of a region edge."""
        if self._smi is not None:
            self.marks[name] = self._accumulators()

    def stop(self) -> None:
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout=2)

    def summary(self, start: str, end: str, flops: Optional[float] = None) -> Dict[str, Any]:
        """Clock / power / temperature spread over the samples between two marks, energy and throttle residency
        over the same interval.  Keys are flat so a bench JSON line carries them directly."""
        if self._smi is None:
            return {"telemetry": f"unavailable ({self.error})"}
        a, b = self.marks.get(start), self.marks.get(end)
        if a is None or b is None:
            return {"telemetry": "region marks missing"}
        win = [s for s in self.samples if a["t"] <= s["t"] <= b["t"]]
        out: Dict[str, Any] = {
            "sclk_mhz": _spread([s["sclk"] for s in win if s["sclk"] is not None], 0),
            "sclk_min_xcd_mhz": _spread([s["sclk_min_xcd"] for s in win if s["sclk_min_xcd"] is not None], 0),
            "power_w": _spread([s["power"] for s in win if s["power"] is not None], 0),
            "temp_hotspot_c": _spread([s["temp_hot"] for s in win if s["temp_hot"] is not None], 0),
            "temp_hbm_c": _spread([s["temp_mem"] for s in win if s["temp_mem"] is not None], 0),
        }
        dt = b["t"] - a["t"]
        if "energy_j" in a and "energy_j" in b and dt > 0:
            ej = b["energy_j"] - a["energy_j"]
            out["energy_j"] = round(ej, 1)
            out["avg_power_w"] = round(ej / dt, 1)
            if flops:
                out["tflop_per_joule"] = round(flops / ej / 1e12, 4) if ej > 0 else None
        if "accumulation_counter" in a and "accumulation_counter" in b:
            n = b["accumulation_counter"] - a["accumulation_counter"]
            if n > 0:
                for k, key in (("ppt_residency_acc", "ppt_limited_frac"), ("socket_thm_residency_acc", "thermal_limited_frac"),
                               ("prochot_residency_acc", "prochot_frac"), ("hbm_thm_residency_acc", "hbm_thermal_frac")):
                    if k in a and k in b:
                        out[key] = round(max(0, b[k] - a[k]) / n, 4)
        return out

"""Graph-replay timeline of one decode token (llmi_engine_debug_timeline): every stamped
launch of the captured step records {start, end, CU} per workgroup with the 100 MHz
s_memrealtime clock into its own region, so one replay reports each kernel's span
(first workgroup start -> last workgroup end) and the gap to the next launch. Used by
tools/graph_timeline.py and bench.py's side measurement (rocprofv3 cannot trace graph
replays on this image)."""
import ctypes as C

import numpy as np

from . import _lib

KINDS = ("qkv", "attn", "o", "gate_up", "down")


def analyse(host, n_slots, stride, layers):
    spans, starts, ends, names = [], [], [], []
    for s in range(n_slots):
        rows = host[s * stride:(s + 1) * stride]
        v = rows[rows[:, 0] > 0].astype(np.int64)
        if not len(v):
            continue
        names.append(KINDS[s % 5] if s < 5 * layers else "lm_head")
        starts.append(v[:, 0].min())
        ends.append(v[:, 3].max())
    starts, ends = np.array(starts), np.array(ends)
    t0 = starts[0]
    span = (ends - starts) / 100.0
    gap = (starts[1:] - ends[:-1]) / 100.0
    out = {"launches": len(names), "token_us_first_start_to_last_end": round(float((ends[-1] - t0) / 100.0), 1),
           "sum_spans_us": round(float(span.sum()), 1), "sum_gaps_us": round(float(gap.sum()), 1)}
    per = {}
    for k in KINDS + ("lm_head",):
        idx = [i for i, n in enumerate(names) if n == k]
        if not idx:
            continue
        g = [gap[i] for i in idx if i < len(gap)]
        per[k] = {"n": len(idx), "span_us_mean": round(float(span[idx].mean()), 2),
                  "span_us_min": round(float(span[idx].min()), 2), "span_us_max": round(float(span[idx].max()), 2),
                  "gap_after_us_mean": round(float(np.mean(g)), 2) if g else None}
    out["per_kernel"] = per
    out["gap_us_quantiles"] = [round(float(x), 2) for x in np.quantile(gap, [0, 0.1, 0.5, 0.9, 1.0])]
    return out



def slot_wgs(cfg) -> int:
    """Workgroups per launch region: the largest decode grid (llmi_engine_debug_timeline)."""
    ns = (cfg.max_seq + 63) // 64
    return max(1024, cfg.heads * ns, cfg.heads * ((cfg.hidden + 15) // 16))


def stamped_token(eng, n_prior: int):
    """Replay n_prior graph tokens unstamped-equivalent, then ONE stamped token; returns
    analyse()'s summary. The engine must have a prompt set at position 0."""
    lib = _lib.lib()
    cfg = eng.cfg
    stride = slot_wgs(cfg)
    n_slots = 5 * cfg.layers + 1
    nbytes = n_slots * stride * 64
    buf = C.c_void_p()
    _lib.call("llmi_device_alloc", C.byref(buf), C.c_size_t(nbytes))
    try:
        _lib.call("llmi_engine_debug_timeline", eng._h, buf, C.c_size_t(nbytes), stride)
        if n_prior:
            eng.decode(n_prior)
        eng.sync()
        _lib.call("llmi_device_memset", buf, 0, C.c_size_t(nbytes))
        eng.decode(1)
        eng.sync()
        host = np.zeros((n_slots * stride, 8), np.uint64)
        _lib.call("llmi_memcpy", host.ctypes.data_as(C.c_void_p), buf, C.c_size_t(nbytes), 1)
        return analyse(host, n_slots, stride, cfg.layers)
    finally:
        lib.llmi_engine_debug_timeline(eng._h, None, C.c_size_t(0), 0)
        lib.llmi_device_free(buf)

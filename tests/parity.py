"""GPU-vs-oracle column comparison (bit-exact for every integer, decimal, float and string)."""
from __future__ import annotations

from typing import List

import numpy as np

from cobrix_amd import native as N
from oracle import oracle as O


def compare_batch(batch, res: "O.OracleResult", max_report: int = 10) -> List[str]:
    plan = batch.plan
    ocols = O.columns(res)
    errs: List[str] = []
    n_rec = batch.n_rec
    if n_rec != res.n_rec:
        return [f"record count {n_rec} != oracle {res.n_rec}"]
    for ci, info in enumerate(plan.columns):
        if info.kind not in ("value", "count") or info.hidden:
            continue
        nid = res.ast.node_of(info.node)
        g = batch.host_column(ci)
        o = ocols.get(nid)
        if info.kind == "count":
            got = g["values"][:n_rec].astype(np.int64)
            if o is None:
                continue
            # count of the top-level occurrence (slot 0 of the enclosing arrays)
            sel = o["slot"] == 0
            exp = np.full(n_rec, -1, dtype=np.int64)
            exp[o["rec"][sel]] = o["count"][sel]
            known = exp >= 0
            bad = np.nonzero(known & (got != exp))[0]
            if len(bad):
                errs.append(f"{info.node.name} counts differ at records {bad[:5]}: {got[bad[:5]]} vs {exp[bad[:5]]}")
            continue
        exp_valid = np.zeros((info.n_slots, n_rec), dtype=bool)
        if o is not None:
            exp_valid[o["slot"], o["rec"]] = o["valid"]
        gv = g["validity"]
        bad = np.argwhere(gv != exp_valid)
        if len(bad):
            s, r = bad[0]
            errs.append(f"{info.node.name}: validity differs at {len(bad)} values, first slot {s} record {r}: "
                        f"gpu {gv[s, r]} oracle {exp_valid[s, r]}")
            continue
        if o is None:
            continue
        m = o["valid"]
        rec, slot = o["rec"][m], o["slot"][m]
        v = slot * n_rec + rec
        ot = info.out_type
        if ot in (N.O_STRING, N.O_BINARY):
            heap = res.heap
            lo, hi = o["lo"][m], o["hi"][m]
            nbad = 0
            for k in range(len(v)):
                if "strings" in g:   # string-view layout, decoded by host_column
                    a = g["strings"][slot[k]][rec[k]]
                else:
                    so = g["offsets"][slot[k]]   # per-slot Arrow offsets (absolute into data)
                    a = g["data"][int(so[rec[k]]):int(so[rec[k] + 1])]
                b = heap[int(lo[k]):int(lo[k]) + int(hi[k])]
                if a != b:
                    nbad += 1
                    if nbad <= 3:
                        errs.append(f"{info.node.name}: string differs at record {rec[k]} slot {slot[k]}: {a!r} vs {b!r}")
            continue
        vals = g["values"]
        lo = o["lo"][m].astype(np.int64)
        hi = o["hi"][m].astype(np.int64)
        if ot == N.O_I32:
            got = vals[v].astype(np.int64)
            exp = lo.astype(np.int32).astype(np.int64)
            diff = got != exp
        elif ot in (N.O_I64, N.O_DEC64):
            diff = vals[v].astype(np.int64) != lo
        elif ot == N.O_DEC128:
            diff = (vals[v, 0].astype(np.int64) != lo) | (vals[v, 1].astype(np.int64) != hi)
        elif ot == N.O_F32:
            diff = (vals[v].astype(np.int64) & 0xFFFFFFFF) != (lo & 0xFFFFFFFF)
        else:
            diff = vals[v].astype(np.int64) != lo
        idx = np.nonzero(diff)[0]
        if len(idx):
            k = idx[0]
            errs.append(f"{info.node.name}: {len(idx)} values differ, first record {rec[k]} slot {slot[k]}: "
                        f"gpu {vals[v[k]]} oracle lo={lo[k]} hi={hi[k]}")
        if len(errs) >= max_report:
            break
    return errs


def compare_sample(batch, idx: np.ndarray, res: "O.OracleResult", max_report: int = 10) -> List[str]:
    """Like compare_batch for a sample of a (large) device batch: res holds the oracle's decode of
    the records idx (in that order); every value of those records is gathered on the device and
    compared bit for bit (validity, fixed-width values, string bytes)."""
    import torch
    plan = batch.plan
    ocols = O.columns(res)
    errs: List[str] = []
    n = batch.n_rec
    pitch = 64 * ((n + 63) // 64)
    words = pitch // 64
    dev_idx = torch.as_tensor(idx, dtype=torch.int64, device=batch.cols[0]["validity"].device)
    for ci, info in enumerate(plan.columns):
        if info.kind != "value" or info.hidden or info.list_array >= 0:   # lists: compare_sample_lists
            continue
        c = batch.cols[ci]
        o = ocols.get(res.ast.node_of(info.node))
        exp_valid = np.zeros((info.n_slots, len(idx)), dtype=bool)
        if o is not None:
            exp_valid[o["slot"], o["rec"]] = o["valid"]
        vw = c["validity"].view(info.n_slots, words)
        for s in range(info.n_slots):
            w = vw[s, dev_idx // 64]
            got_valid = ((w >> (dev_idx % 64)) & 1).cpu().numpy().astype(bool)
            if not np.array_equal(got_valid, exp_valid[s]):
                k = int(np.nonzero(got_valid != exp_valid[s])[0][0])
                errs.append(f"{info.node.name}[{s}]: validity differs at record {idx[k]}")
        if o is None:
            continue
        m = o["valid"]
        rec, slot = o["rec"][m], o["slot"][m]
        ot = info.out_type
        if ot in (N.O_STRING, N.O_BINARY):
            views = c["views"].view(info.n_slots, pitch, 16) if "views" in c else None
            if views is not None:
                offs = None
            elif "offsets32" in c:   # Utf8: relative to the slot's region
                offs = (c["offsets32"].view(info.n_slots, pitch + 1).to(torch.int64) +
                        c["capacity"] * torch.arange(info.n_slots, device=c["offsets32"].device).view(-1, 1))
            else:
                offs = c["offsets"].view(info.n_slots, pitch + 1)
            for k in range(len(rec)):
                r, s = int(idx[rec[k]]), int(slot[k])
                if views is not None:
                    vb = views[s, r].cpu().numpy()
                    ln, bi, of = (int(x) for x in vb.view(np.int32)[[0, 2, 3]])
                    if ln <= 12:
                        got = bytes(vb[4:4 + ln])
                    else:
                        a0 = s * c["capacity"] + bi * c["buffer_bytes"] + of
                        got = bytes(c["data"][a0:a0 + ln].cpu().numpy())
                        if got[:4] != bytes(vb[4:8]):
                            errs.append(f"{info.node.name}: view prefix differs at record {r}")
                            break
                else:
                    a0, a1 = int(offs[s, r]), int(offs[s, r + 1])
                    got = bytes(c["data"][a0:a1].cpu().numpy())
                want = res.heap[int(o["lo"][m][k]):int(o["lo"][m][k]) + int(o["hi"][m][k])]
                if got != want:
                    errs.append(f"{info.node.name}: string differs at record {r}: {got!r} vs {want!r}")
                    break
            continue
        w = N.OUT_WIDTH[ot]
        vals = c["values"]
        pos = torch.as_tensor(slot * pitch + idx[rec], dtype=torch.int64, device=vals.device)
        lo = o["lo"][m].astype(np.int64)
        if ot == N.O_DEC128:
            v2 = vals.view(-1, 2)[pos].cpu().numpy()
            bad = (v2[:, 0] != lo) | (v2[:, 1] != o["hi"][m].astype(np.int64))
        elif w == 4:
            got = vals.view(-1)[pos].cpu().numpy().astype(np.int64) & 0xFFFFFFFF
            bad = got != (lo & 0xFFFFFFFF)
        else:
            bad = vals.view(-1)[pos].cpu().numpy().astype(np.int64) != lo
        if bad.any():
            k = int(np.nonzero(bad)[0][0])
            errs.append(f"{info.node.name}: {int(bad.sum())} values differ, first record {idx[rec[k]]}")
        if len(errs) >= max_report:
            break
    return errs


def compare_sample_lists(batch, idx: np.ndarray, res: "O.OracleResult", max_report: int = 10) -> List[str]:
    """compare_sample for the list-layout columns (OCCURS DEPENDING ON elements packed per record):
    for every sampled record its element count, list offset and the values + validity of its present
    elements, gathered on the device, against the oracle's decode of those records."""
    import torch
    plan = batch.plan
    ocols = O.columns(res)
    errs: List[str] = []
    dev = batch.cols[0]["validity"].device
    di = torch.as_tensor(idx, dtype=torch.int64, device=dev)
    for ci, info in enumerate(plan.columns):
        if info.list_array < 0 or info.kind != "value" or info.hidden:
            continue
        ar = plan.arrays[info.list_array]
        cnt = batch.cols[ar.count_column]["values"][di].to(torch.int64)
        cv = batch.cols[ar.count_column]["validity"]
        cbit = ((cv[di // 64] >> (di % 64)) & 1).bool()
        cnt = torch.where(cbit, cnt, torch.zeros_like(cnt)).cpu().numpy()
        off = batch.cols[ar.offsets_column]["values"][di].to(torch.int64).cpu().numpy()
        o = ocols.get(res.ast.node_of(info.node))
        orec = o["rec"].astype(np.int64) if o is not None else np.zeros(0, np.int64)
        oslot = o["slot"].astype(np.int64) if o is not None else np.zeros(0, np.int64)
        n_exp = np.zeros(len(idx), np.int64)
        np.maximum.at(n_exp, orec, oslot + 1)
        if not np.array_equal(cnt, n_exp):
            k = int(np.nonzero(cnt != n_exp)[0][0])
            errs.append(f"{info.node.name}: element count {cnt[k]} != {n_exp[k]} at record {idx[k]}")
            continue
        if not cnt.sum():
            continue
        pos = np.concatenate([off[k] + np.arange(cnt[k]) for k in range(len(idx))])
        who = np.repeat(np.arange(len(idx)), cnt)
        j = np.concatenate([np.arange(c) for c in cnt])
        tp = torch.as_tensor(pos, dtype=torch.int64, device=dev)
        vbits = ((batch.cols[ci]["validity"][tp // 64] >> (tp % 64)) & 1).bool().cpu().numpy()
        vals = batch.cols[ci]["values"]
        # the oracle's entries in (record, element) order, matched to the gathered elements
        okey = orec * 65536 + oslot
        srt = np.argsort(okey, kind="stable")
        okey, ovalid = okey[srt], o["valid"][srt].astype(bool)
        olo, ohi = o["lo"][srt].astype(np.int64), o["hi"][srt].astype(np.int64)
        gk = who.astype(np.int64) * 65536 + j
        at = np.searchsorted(okey, gk)
        found = (at < len(okey)) & (okey[np.minimum(at, len(okey) - 1)] == gk)
        at = np.minimum(at, len(okey) - 1)
        bad = ~found | (ovalid[at] != vbits)
        both = found & ovalid[at] & vbits
        if info.out_type == N.O_DEC128:
            got = vals.view(-1, 2)[tp].cpu().numpy()
            bad |= both & ((got[:, 0] != olo[at]) | (got[:, 1] != ohi[at]))
        elif N.OUT_WIDTH[info.out_type] == 4:
            got = vals.view(-1)[tp].cpu().numpy().astype(np.int64) & 0xFFFFFFFF
            bad |= both & (got != (olo[at] & 0xFFFFFFFF))
        else:
            got = vals.view(-1)[tp].cpu().numpy().astype(np.int64)
            bad |= both & (got != olo[at])
        bad = int(bad.sum())
        if bad:
            errs.append(f"{info.node.name}: {bad} of {len(pos)} sampled elements differ")
        if len(errs) >= max_report:
            break
    return errs

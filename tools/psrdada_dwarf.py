#!/usr/bin/env python3
"""Extract PSRDADA's ABI from the reference's own binaries -> tests/golden/psrdada_abi.json.

The reference links libpsrdada statically, with debug info, into its three
shipped executables.  This script reads that debug
info as text (`readelf --debug-dump=info`; the binaries are never run or
loaded) and records, for the PSRDADA subset libpafdada implements:

  * the struct layouts: ipcsync_t (the shared sync segment), ipcbuf_t,
    ipcio_t, dada_hdu_t -- member names, offsets, sizes, C types;
  * the prototypes of the ipcbuf_* / ipcio_* / dada_hdu_* / multilog* /
    ascii_header_* / fileread functions (return and parameter types);
  * the ring protocol read off the disassembly (`objdump -d -l`) of the same
    functions: the SysV key schedule, the semaphore sets and their initial
    values, the reader/writer state numbers.  These are recorded by hand in
    PROTOCOL below, each with the instruction addresses they come from, and
    the script checks every address still names the function it cites.

The JSON is a fixture (data), committed so the CPU tests can pin
libpafdada's shared-memory layout and the PSRDADA stand-in headers to it
without /root/reference.  Usage:  python tools/psrdada_dwarf.py [--check]
"""
from __future__ import annotations

import json
import os
import re
import subprocess
import sys

REF = "/root/reference"
BINARIES = ("paf_diskdb", "paf_capture", "paf_baseband2power")
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests", "golden",
                   "psrdada_abi.json")
STRUCTS = {"ipcsync_t", "ipcbuf_t", "ipcio_t", "dada_hdu"}
FUNC_RE = re.compile(r"^(ipcbuf_|ipcio_|dada_hdu_|multilog|ascii_header_|fileread$|ipc_alloc$|ipc_semop$)")

# ---- protocol facts from the disassembly of paf_diskdb (objdump -d -l) ----------
# addr -> the function it lies in (checked against the symbol table below)
PROTOCOL = {
    "ipcsync_segment": {
        "what": "shmget(key, 520 + 5*nbufs): ipcsync_t, then char count[nbufs], then "
                "key_t shmkey[nbufs] (ipcsync_get: lea 0x208(%rdx,%rdx,4); count = sync+0x208, "
                "shmkey = count+nbufs)",
        "size": "520 + 5*nbufs", "count_offset": 520, "shmkey_offset": "520 + nbufs",
        "evidence": [["ipcsync_get", "0x402fea"], ["ipcsync_get", "0x403014"],
                     ["ipcsync_get", "0x403028"]],
    },
    "keys": {
        "what": "semkey_connect = key + 0x10000; semkey_data[i] = key + 0x10000*(2+i), i < 8; "
                "shmkey[ibuf] = key + 0x10000*(10+ibuf)",
        "semkey_connect": 0x10000, "semkey_data_step": 0x10000, "semkey_data_first": 0x20000,
        "shmkey_first": 0xA0000, "shmkey_step": 0x10000,
        "evidence": [["ipcbuf_create_work", "0x40344a"], ["ipcbuf_create_work", "0x403460"],
                     ["ipcbuf_create_work", "0x403484"]],
    },
    "create_flags": {"create": 0o3666, "connect": 0o666,
                     "evidence": [["ipcbuf_create_work", "0x4033bb"], ["ipcbuf_connect", "0x4036f3"]]},
    "sem_connect": {
        "what": "semget(semkey_connect, 2): [0] IPCBUF_WRITE = 1 (writer lock), "
                "[1] IPCBUF_READ = n_readers",
        "nsems": 2, "WRITE": 0, "READ": 1, "init": {"WRITE": 1, "READ": "n_readers"},
        "evidence": [["ipcbuf_get", "0x4030b3"], ["ipcbuf_create_work", "0x403528"],
                     ["ipcbuf_create_work", "0x403541"]],
    },
    "sem_data": {
        "what": "semget(semkey_data[i], 5) for i < n_readers: [0] SODACK = 8, [1] EODACK = 8, "
                "[2] FULL = 0, [3] CLEAR = 0, [4] READER_CONN = 1",
        "nsems": 5, "SODACK": 0, "EODACK": 1, "FULL": 2, "CLEAR": 3, "READER_CONN": 4,
        "init": {"SODACK": 8, "EODACK": 8, "FULL": 0, "CLEAR": 0, "READER_CONN": 1},
        "evidence": [["ipcbuf_get", "0x403129"], ["ipcbuf_create_work", "0x4035c2"],
                     ["ipcbuf_create_work", "0x403578"], ["ipcbuf_create_work", "0x403598"]],
    },
    "create_sync_init": {
        "what": "for x < 8: s_buf = s_byte = e_buf = e_byte = 0, eod[x] = 1; w_buf = w_xfer = "
                "w_state = 0; r_bufs = r_xfers = r_states = 0",
        "evidence": [["ipcbuf_create_work", "0x403408"], ["ipcbuf_create_work", "0x403434"],
                     ["ipcbuf_create_work", "0x4034a1"], ["ipcbuf_create_work", "0x4034c0"]],
    },
    "states": {
        "DISCON": 0, "VIEWER": 1, "WRITER": 2, "WRITING": 3, "WCHANGE": 4, "READER": 5,
        "READING": 6, "RSTOP": 7, "VIEWING": 8, "VSTOP": 9,
        "evidence": [["ipcbuf_lock_write", "0x403b25"], ["ipcbuf_enable_eod", "0x403c20"],
                     ["ipcbuf_lock_read", "0x4044e5"], ["ipcbuf_mark_cleared", "0x404bf6"],
                     ["ipcbuf_get_next_read_work", "0x404887"], ["ipcbuf_eod", "0x405247"]],
    },
    "write_protocol": {
        "lock_write": "semop(connect, WRITE, -1, SEM_UNDO); state = w_state ? WRITING : WCHANGE; "
                      "xfer = w_xfer % 8",
        "get_next_write": "WCHANGE -> enable_sod(w_buf, 0); b = w_buf % nbufs; while count[b]: "
                          "semop(data[r], CLEAR, -1) for every reader, count[b]--",
        "enable_sod": "for every reader semop(data[r], SODACK, -1); xfer = w_xfer % 8; "
                      "s_buf/s_byte[xfer] = start; w_buf == 0 ? eod[xfer] = 0 : count[b]++ for "
                      "b in [start_buf, w_buf); state = w_state = WRITING; FULL += w_buf - s_buf",
        "mark_filled": "WRITER: w_buf++ only.  WCHANGE or nbytes < bufsz: semop(data[r], "
                       "EODACK, -1) per reader, e_buf[xfer] = w_buf, e_byte[xfer] = nbytes, "
                       "eod[xfer] = 1, w_xfer++, state = WRITER, w_state = 0.  Then "
                       "count[w_buf % nbufs]++, w_buf++, semop(data[r], FULL, +1) per reader",
        "enable_eod": "WRITING -> WCHANGE (the next mark_filled ends the transfer)",
        "ipcio_close": "writer WRITING: enable_eod + mark_filled(bytes written into the open "
                       "block, 0 if none) -- a 0-byte EOD block when the last block was full",
        "evidence": [["ipcbuf_lock_write", "0x403b09"], ["ipcbuf_get_next_write", "0x403f6c"],
                     ["ipcbuf_get_next_write", "0x403fb1"], ["ipcbuf_enable_sod", "0x403d57"],
                     ["ipcbuf_enable_sod", "0x403dda"], ["ipcbuf_enable_sod", "0x403e34"],
                     ["ipcbuf_mark_filled", "0x404268"], ["ipcbuf_mark_filled", "0x40428d"],
                     ["ipcbuf_mark_filled", "0x4041e2"], ["ipcbuf_mark_filled", "0x40421d"],
                     ["ipcio_stop_close", "0x405ce8"], ["ipcio_stop_close", "0x405cf8"]],
    },
    "read_protocol": {
        "lock_read": "semop(connect, READ, -1, SEM_UNDO); take the free reader slot with the "
                     "lowest r_bufs (semop(data[r], READER_CONN, -1, IPC_NOWAIT|SEM_UNDO)); "
                     "state = r_states[r] ? READING : READER; xfer = r_xfers[r] % 8",
        "get_next_read": "RSTOP -> NULL; semop(data[r], FULL, -1); READER: xfer = r_xfers % 8, "
                         "state = r_states = READING, r_bufs = s_buf[xfer], start = s_byte[xfer], "
                         "semop(data[r], SODACK, +1); bytes = (eod[xfer] && e_buf[xfer] == "
                         "r_bufs) ? e_byte - start : bufsz - start",
        "mark_cleared": "semop(data[r], CLEAR, +1); eod[xfer] && r_bufs == e_buf[xfer] ? "
                        "(state = RSTOP, r_states = 0, r_xfers++, semop(data[r], EODACK, +1)) "
                        ": r_bufs++",
        "reset": "reader RSTOP -> READER (the next transfer)",
        "unlock_read": "semop(data[r], READER_CONN, +1, SEM_UNDO); semop(connect, READ, +1, "
                       "SEM_UNDO)",
        "evidence": [["ipcbuf_lock_read", "0x404394"], ["ipcbuf_lock_read", "0x404498"],
                     ["ipcbuf_get_next_read_work", "0x404852"],
                     ["ipcbuf_get_next_read_work", "0x404939"],
                     ["ipcbuf_get_next_read_work", "0x4047e7"], ["ipcbuf_mark_cleared", "0x404b91"],
                     ["ipcbuf_mark_cleared", "0x404c11"], ["ipcbuf_reset", "0x404df8"],
                     ["ipcbuf_unlock_read", "0x404616"], ["ipcbuf_unlock_read", "0x404639"]],
    },
    "view_protocol": {
        "open": "ipcio_open 'r': no lock, rdwrt = 'r'; ipcio_read / open_block_read accept "
                "(rdwrt & ~0x20) == 'R'; only 'R' calls mark_cleared",
        "first_view": "VIEWER -> VIEWING: xfer = r_xfers[0] % 8, viewbuf = s_buf[xfer]; "
                      "w_buf > s_buf + 1 ? viewbuf = w_buf - 1 (the newest block), start 0 : "
                      "start = s_byte[xfer]",
        "next": "while w_buf <= viewbuf: eod[xfer] && r_bufs[0] && r_bufs[0] == e_buf[xfer] "
                "-> VSTOP, else float_sleep(0.1); viewbuf + nbufs < w_buf -> viewbuf = "
                "w_buf - nbufs + 1 (lapped); block = viewbuf++",
        "evidence": [["ipcio_open", "0x405a48"], ["ipcbuf_get_next_read_work", "0x404880"],
                     ["ipcbuf_get_next_read_work", "0x4048f4"],
                     ["ipcbuf_get_next_read_work", "0x4048c0"],
                     ["ipcbuf_get_next_read_work", "0x40479d"],
                     ["ipcbuf_get_next_read_work", "0x404820"], ["ipcio_read", "0x406776"]],
    },
    "deferred_start": {
        "open": "ipcio_open 'w': lock_write + disable_sod (WRITER: mark_filled only w_buf++)",
        "start": "ipcio_start(byte) needs rdwrt 'w': sod_pending = 1, rdwrt = 'W', sod_buf = "
                 "byte / bufsz, sod_byte = byte % bufsz, then check_pending_sod",
        "check_pending_sod": "sod_pending && w_buf > sod_buf -> enable_sod(sod_buf, sod_byte), "
                             "sod_pending = 0",
        "stop_close": "'W' writing: enable_eod, mark_filled(bytes), check_pending_sod, "
                      "marked_filled = 1, curbuf = 0 if bytes == bufsz; rdwrt = 'w'; unlock: "
                      "w_xfer ? w_buf = e_buf[(w_xfer-1) % 8] + 1, unlock_write",
        "evidence": [["ipcio_open", "0x405a19"], ["ipcio_start", "0x405bb8"],
                     ["ipcio_check_pending_sod", "0x405b5a"], ["ipcio_stop_close", "0x405c81"],
                     ["ipcio_stop", "0x405ddb"], ["ipcio_close", "0x405e10"]],
    },
    "resets": {
        "reset_writer": "writer with w_buf > 0: CLEAR -1 per reader for every count[], SODACK and "
                        "EODACK -8 then +8 per reader, r_bufs = r_xfers = 0, w_buf = w_xfer = 0, "
                        "eod[] = 1",
        "hard_reset": "w_buf = w_xfer = 0, eod[] = 1, per reader r_bufs = r_xfers = 0 and "
                      "semctl SETVAL 0 of FULL and CLEAR (count[] untouched)",
        "evidence": [["ipcbuf_reset", "0x404d60"], ["ipcbuf_reset", "0x404e43"],
                     ["ipcbuf_reset", "0x404d98"], ["ipcbuf_hard_reset", "0x40501f"],
                     ["ipcbuf_hard_reset", "0x404fdd"]],
    },
    "device_blocks": {
        "what": "on_device_id >= 0: block ibuf's segment at shmkey[ibuf] holds a 64-B IPC memory "
                "handle (ipc_alloc_cuda: shmget(key, 64); creator allocates and publishes the "
                "handle, others open it)",
        "handle_bytes": 64,
        "evidence": [["ipc_alloc_cuda", "0x407ede"], ["ipc_alloc_cuda", "0x407fd8"],
                     ["ipc_alloc_cuda", "0x407f3d"]],
    },
}


def readelf(path: str) -> str:
    return subprocess.run(["readelf", "--debug-dump=info", path], capture_output=True, text=True,
                          check=True).stdout


DIE_RE = re.compile(r"^\s*<(\d+)><([0-9a-f]+)>: Abbrev Number: \d+ \((DW_TAG_\w+)\)")
ATTR_RE = re.compile(r"^\s*<[0-9a-f]+>\s+(DW_AT_\w+)\s*:\s*(.*)$")


def parse_dies(text: str):
    """flat list of DIEs: dict(off, depth, tag, attrs, children[]) with tree links"""
    dies, stack = {}, []
    roots = []
    cur = None
    for line in text.splitlines():
        m = DIE_RE.match(line)
        if m:
            depth, off, tag = int(m.group(1)), int(m.group(2), 16), m.group(3)
            cur = {"off": off, "depth": depth, "tag": tag, "attrs": {}, "children": []}
            dies[off] = cur
            while stack and stack[-1]["depth"] >= depth:
                stack.pop()
            if stack:
                stack[-1]["children"].append(cur)
            else:
                roots.append(cur)
            stack.append(cur)
            continue
        m = ATTR_RE.match(line)
        if m and cur is not None:
            val = m.group(2).strip()
            if "(indirect string" in val:
                val = val.split("):", 1)[1].strip()
            cur["attrs"][m.group(1)] = val
    return dies, roots


def member_offset(v: str) -> int:
    """DW_AT_data_member_location: a constant, or (older producers, the
    nvcc-compiled units) a DW_OP_plus_uconst expression"""
    m = re.search(r"DW_OP_plus_uconst: (\d+)", v)
    return int(m.group(1)) if m else int(v)


def ref(v: str) -> int:
    return int(v.strip().strip("<>"), 16)


class TypeNamer:
    def __init__(self, dies):
        self.d = dies

    def name(self, off) -> str:
        if off is None:
            return "void"
        die = self.d[off]
        t, a = die["tag"], die["attrs"]
        sub = ref(a["DW_AT_type"]) if "DW_AT_type" in a else None
        if t in ("DW_TAG_base_type", "DW_TAG_typedef"):
            return a.get("DW_AT_name", "?")
        if t == "DW_TAG_structure_type":
            return "struct " + a.get("DW_AT_name", "<anon>")
        if t == "DW_TAG_pointer_type":
            return self.name(sub) + " *"
        if t == "DW_TAG_const_type":
            return "const " + self.name(sub)
        if t in ("DW_TAG_restrict_type", "DW_TAG_volatile_type"):
            return self.name(sub)
        if t == "DW_TAG_array_type":
            dims = [int(c["attrs"].get("DW_AT_upper_bound", "-1")) + 1 for c in die["children"]
                    if c["tag"] == "DW_TAG_subrange_type"]
            return self.name(sub) + "".join(f"[{n}]" for n in dims)
        if t == "DW_TAG_subroutine_type":
            return "fnptr"
        return t

    def size(self, off) -> int:
        die = self.d[off]
        a = die["attrs"]
        if "DW_AT_byte_size" in a:
            return int(a["DW_AT_byte_size"])
        if die["tag"] in ("DW_TAG_typedef", "DW_TAG_const_type", "DW_TAG_volatile_type"):
            return self.size(ref(a["DW_AT_type"]))
        if die["tag"] == "DW_TAG_array_type":
            n = 1
            for c in die["children"]:
                if c["tag"] == "DW_TAG_subrange_type":
                    n *= int(c["attrs"].get("DW_AT_upper_bound", "-1")) + 1
            return n * self.size(ref(a["DW_AT_type"]))
        return -1


def extract(path: str):
    dies, roots = parse_dies(readelf(path))
    tn = TypeNamer(dies)
    structs, funcs = {}, {}
    for die in dies.values():
        a = die["attrs"]
        if die["tag"] == "DW_TAG_typedef" and a.get("DW_AT_name") in STRUCTS | {"dada_hdu_t"}:
            sdie = dies[ref(a["DW_AT_type"])]
            name = a["DW_AT_name"]
        elif die["tag"] == "DW_TAG_structure_type" and a.get("DW_AT_name") in STRUCTS:
            sdie, name = die, a["DW_AT_name"]
        else:
            sdie = None
        if sdie is not None and sdie["tag"] == "DW_TAG_structure_type" and sdie["children"]:
            name = "dada_hdu_t" if name == "dada_hdu" else name
            members = []
            for m in sdie["children"]:
                if m["tag"] != "DW_TAG_member":
                    continue
                t = ref(m["attrs"]["DW_AT_type"])
                members.append({"name": m["attrs"]["DW_AT_name"],
                                "offset": member_offset(m["attrs"]["DW_AT_data_member_location"]),
                                "size": tn.size(t), "type": tn.name(t)})
            structs[name] = {"size": int(sdie["attrs"]["DW_AT_byte_size"]), "members": members}
        decl = die
        if die["tag"] == "DW_TAG_subprogram" and "DW_AT_abstract_origin" in a:
            decl = dies[ref(a["DW_AT_abstract_origin"])]  # out-of-line copy of an inline
        da = decl["attrs"]
        if die["tag"] == "DW_TAG_subprogram" and FUNC_RE.match(da.get("DW_AT_name", "")) and \
                "DW_AT_low_pc" in a:
            a = da
            ret = tn.name(ref(a["DW_AT_type"])) if "DW_AT_type" in a else "void"
            params = []
            for c in decl["children"]:
                if c["tag"] == "DW_TAG_formal_parameter":
                    params.append({"name": c["attrs"].get("DW_AT_name", ""),
                                   "type": tn.name(ref(c["attrs"]["DW_AT_type"]))})
                elif c["tag"] == "DW_TAG_unspecified_parameters":
                    params.append({"name": "...", "type": "..."})
            funcs[a["DW_AT_name"]] = {"return": ret, "params": params,
                                      "low_pc": die["attrs"]["DW_AT_low_pc"]}
    return structs, funcs


def symbols(path: str):
    out = subprocess.run(["nm", path], capture_output=True, text=True, check=True).stdout
    syms = []
    for line in out.splitlines():
        p = line.split()
        if len(p) == 3 and p[1] in "tT":
            syms.append((int(p[0], 16), p[2]))
    syms.sort()
    return syms


def func_at(syms, addr: int) -> str:
    best = None
    for a, n in syms:
        if a <= addr:
            best = n
        else:
            break
    return best.split(".")[0] if best else ""


def build():
    structs, funcs, seen_in = {}, {}, {}
    for b in BINARIES:
        s, f = extract(os.path.join(REF, b))
        for k, v in s.items():
            if k in structs and structs[k] != v:
                raise SystemExit(f"{k} differs between binaries")
            structs[k] = v
            seen_in.setdefault(k, []).append(b)
        for k, v in f.items():
            v = dict(v)
            lp = v.pop("low_pc")
            if k in funcs and (funcs[k]["return"], funcs[k]["params"]) != (v["return"], v["params"]):
                raise SystemExit(f"{k} prototype differs between binaries")
            funcs.setdefault(k, v)
            funcs[k].setdefault("low_pc", {})[b] = lp
    syms = symbols(os.path.join(REF, "paf_diskdb"))
    for key, fact in PROTOCOL.items():
        for fn, addr in fact.get("evidence", []):
            got = func_at(syms, int(addr, 16))
            if got != fn:
                raise SystemExit(f"PROTOCOL[{key}]: {addr} lies in {got}, not {fn}")
    return {
        "source": "DWARF (readelf --debug-dump=info) and disassembly (objdump -d -l) of the "
                  "reference's statically linked libpsrdada in " + ", ".join(BINARIES) +
                  "; generated by tools/psrdada_dwarf.py",
        "structs": structs, "struct_binaries": seen_in,
        "functions": dict(sorted(funcs.items())),
        "protocol": PROTOCOL,
    }


def main():
    data = build()
    text = json.dumps(data, indent=1, sort_keys=False) + "\n"
    if "--check" in sys.argv:
        old = open(OUT).read()
        if old != text:
            raise SystemExit("tests/golden/psrdada_abi.json is stale")
        print("up to date")
        return
    with open(OUT, "w") as f:
        f.write(text)
    print(f"{OUT}: {len(data['structs'])} structs, {len(data['functions'])} functions")


if __name__ == "__main__":
    main()

"""Python host mirror of the nttmul C ABI (include/nttmul.h), over ctypes.

This is the reference-side binding a Python caller uses: it exposes the reference's product entry
points with their names and argument meaning (ntt256_product1/4, ntt_red256_product1/4:
NTT/ntt256.h:85-86, NTT-RED/ntt_red256.h:87,90 — output array c, inputs a, b, n = 256,
q = 12289) plus the generic batched API multiply(a, b) for any (n, q).  All compute runs in
lib/libnttmul.so on the GPU; there is no CPU fallback: if the library or a GPU is missing the calls
raise.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional

import numpy as np

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.path.join(PKG_DIR, "lib", "libnttmul.so")
# the diagnostic build (include/nttmul_diag.h): same kernels plus in-kernel clock stamps
DIAG_LIB_PATH = os.path.join(PKG_DIR, "lib", "libnttmul_diag.so")
HEADER_PATH = os.path.join(os.path.dirname(PKG_DIR), "include", "nttmul.h")

NTTMUL_OK = 0
NTTMUL_EINVAL = -1
NTTMUL_ENODEV = -2
NTTMUL_EHIP = -3
NTTMUL_ENOMEM = -4
NTTMUL_ERANGE = -5
NTTMUL_EUNSUPPORTED = -6
NTTMUL_FLAG_VALIDATE = 1
NTTMUL_FLAG_CYCLIC = 2
NTTMUL_FLAG_SHARE_DEVICES = 4
# transform modes (include/nttmul.h nttmul_transform_*)
XF_FORWARD = 0
XF_INVERSE = 1
XF_STD2REV = 0
XF_REV2STD = 2
XF_UNSCALED = 4
# the reference's n = 256 wrapper set (NTT/ntt256.h:20-69), exported under the same names
NTT256_WRAPPERS = [
    "ntt256_ct_rev2std", "ntt256_gs_rev2std", "ntt256_ct_std2rev", "ntt256_gs_std2rev",
    "intt256_ct_rev2std", "intt256_gs_rev2std", "intt256_ct_std2rev", "intt256_gs_std2rev",
    "mulntt256_ct_rev2std", "mulntt256_ct_std2rev", "inttmul256_gs_rev2std", "inttmul256_gs_std2rev",
]
TABLES = [  # nttmul_table `which` order = the tables of NTT/ntt.h:63-183 (ntt256_tables.h:29-43)
    "psi_powers", "inv_psi_powers", "inv_psi_powers_rev", "scaled_inv_psi_powers",
    "omega_powers", "omega_powers_rev", "inv_omega_powers", "inv_omega_powers_rev",
    "mixed_powers", "mixed_powers_rev", "inv_mixed_powers", "inv_mixed_powers_rev",
]

SEED = 0x4E54544D554C  # "NTTMUL", SURVEY §8d


class NttmulError(RuntimeError):
    def __init__(self, status: int, msg: str):
        super().__init__(f"nttmul status {status}: {msg}")
        self.status = status


class _Params(ctypes.Structure):
    _fields_ = [("n", ctypes.c_uint32), ("q", ctypes.c_uint64), ("psi", ctypes.c_uint64),
                ("ndev", ctypes.c_int), ("first_dev", ctypes.c_int), ("flags", ctypes.c_uint32),
                ("issue_prio", ctypes.c_int32), ("zero_copy_kb", ctypes.c_int32),
                ("copy_threads", ctypes.c_int32), ("scratch_mb", ctypes.c_uint32),
                ("small_server", ctypes.c_int32)]


class Info(ctypes.Structure):
    _fields_ = [("n", ctypes.c_uint32), ("logn", ctypes.c_uint32), ("q", ctypes.c_uint64),
                ("psi", ctypes.c_uint64), ("omega", ctypes.c_uint64),
                ("inv_psi", ctypes.c_uint64), ("inv_omega", ctypes.c_uint64),
                ("inv_n", ctypes.c_uint64), ("word_bits", ctypes.c_uint32),
                ("ndev", ctypes.c_int), ("kernel", ctypes.c_int), ("cyclic", ctypes.c_uint32)]


_LIB: Optional[ctypes.CDLL] = None
_DIAG_LIB: Optional[ctypes.CDLL] = None


def load_library() -> ctypes.CDLL:
    """Load lib/libnttmul.so (built by `make -C ntt-based-polynomial-multiplier-fpga_amd`)."""
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} not built: run __graft_entry__.build() or make -C {PKG_DIR}")
    _LIB = _bind(ctypes.CDLL(LIB_PATH))
    return _LIB


def load_diag_library() -> ctypes.CDLL:
    """Load lib/libnttmul_diag.so (include/nttmul_diag.h): the same ABI, kernels with in-kernel
    clock stamps; used by bench.py for the clock the product kernel holds, never for results."""
    global _DIAG_LIB
    if _DIAG_LIB is not None:
        return _DIAG_LIB
    if not os.path.exists(DIAG_LIB_PATH):
        raise ImportError(f"{DIAG_LIB_PATH} not built")
    lib = _bind(ctypes.CDLL(DIAG_LIB_PATH))
    lib.nttmul_diag_clock_stamps.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    _DIAG_LIB = lib
    return lib


def _bind(lib: ctypes.CDLL) -> ctypes.CDLL:
    vp, sz, u64, u32, i32 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int
    lib.nttmul_create.argtypes = [ctypes.POINTER(vp), u32, u64, i32]
    lib.nttmul_create_ex.argtypes = [ctypes.POINTER(vp), ctypes.POINTER(_Params)]
    lib.nttmul_create_sized.argtypes = [ctypes.POINTER(vp), ctypes.POINTER(_Params), sz]
    lib.nttmul_destroy.argtypes = [vp]
    lib.nttmul_destroy.restype = None
    lib.nttmul_strerror.argtypes = [i32]
    lib.nttmul_strerror.restype = ctypes.c_char_p
    lib.nttmul_last_error.argtypes = [vp]
    lib.nttmul_last_error.restype = ctypes.c_char_p
    lib.nttmul_get_info.argtypes = [vp, ctypes.POINTER(Info)]
    lib.nttmul_kernel_name.argtypes = [vp, i32, ctypes.c_char_p, sz]
    lib.nttmul_kernel_name_batch.argtypes = [vp, i32, sz, ctypes.c_char_p, sz]
    lib.nttmul_last_kernel_name.argtypes = [vp, ctypes.c_char_p, sz]
    lib.nttmul_last_host_path.argtypes = [vp]
    if hasattr(lib, "nttmul_server_status"):  # (round 6; tools/bench_ab.py loads older builds)
        lib.nttmul_server_status.argtypes = [vp, ctypes.c_char_p, sz]
    for name in ("nttmul_multiply_u32", "nttmul_multiply_u64"):
        getattr(lib, name).argtypes = [vp, vp, vp, vp]
    for name in ("nttmul_multiply_batch_u32", "nttmul_multiply_batch_u64"):
        getattr(lib, name).argtypes = [vp, vp, vp, vp, sz]
    lib.nttmul_multiply_batch_device.argtypes = [vp, vp, vp, vp, sz, i32, i32, vp]
    for op in ("forward", "inverse"):
        for w in ("u32", "u64"):
            getattr(lib, f"nttmul_{op}_batch_{w}").argtypes = [vp, vp, vp, sz]
        getattr(lib, f"nttmul_{op}_batch_device").argtypes = [vp, vp, vp, sz, i32, i32, vp]
    for w in ("u32", "u64"):
        getattr(lib, f"nttmul_pointwise_batch_{w}").argtypes = [vp, vp, vp, vp, sz]
    lib.nttmul_pointwise_batch_device.argtypes = [vp, vp, vp, vp, sz, i32, i32, vp]
    lib.nttmul_fill_random_device.argtypes = [vp, vp, vp, u64, sz, u64, i32, i32, vp]
    lib.nttmul_is_prime.argtypes = [u64]
    lib.nttmul_smallest_psi.argtypes = [u32, u64]
    lib.nttmul_smallest_psi.restype = u64
    lib.nttmul_smallest_omega.argtypes = [u32, u64]
    lib.nttmul_smallest_omega.restype = u64
    lib.nttmul_find_prime.argtypes = [u32, i32, i32, ctypes.POINTER(u64)]
    lib.nttmul_table.argtypes = [u32, u64, u64, i32, vp]
    lib.nttmul_fpga_R.argtypes = [u32, i32]
    lib.nttmul_fpga_R.restype = u64
    lib.nttmul_fpga_twiddles.argtypes = [u32, u64, u64, u64, u32, vp, sz]
    lib.nttmul_fpga_twiddles.restype = sz
    lib.nttmul_read_coefficients.argtypes = [ctypes.c_char_p, vp, i32]
    lib.nttmul_read_hex.argtypes = [ctypes.c_char_p, vp, i32]
    lib.nttmul_write_hex.argtypes = [ctypes.c_char_p, vp, i32]
    lib.nttmul_print_array.argtypes = [vp, vp, i32]
    for name in ("ntt256_product1", "ntt256_product4", "ntt_red256_product1", "ntt_red256_product4"):
        getattr(lib, name).argtypes = [vp, vp, vp]
        getattr(lib, name).restype = None
    for w in ("u32", "u64"):
        getattr(lib, f"nttmul_transform_batch_{w}").argtypes = [vp, u32, vp, vp, sz]
    lib.nttmul_transform_device.argtypes = [vp, u32, vp, vp, sz, i32, i32, vp]
    for name in NTT256_WRAPPERS:
        getattr(lib, name).argtypes = [vp]
        getattr(lib, name).restype = None
    return lib


def _elf_sections(elf: bytes) -> dict:
    """{section name: bytes} of an ELF64 image (NOBITS sections map to b"")."""
    import struct
    if elf[:4] != b"\x7fELF" or elf[4] != 2:
        raise ValueError("not an ELF64 image")
    shoff, = struct.unpack_from("<Q", elf, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", elf, 0x3A)

    def sec(i):
        return struct.unpack_from("<IIQQQQ", elf, shoff + i * shentsize)
    stroff = sec(shstrndx)[4]
    out = {}
    for i in range(shnum):
        name, typ, _, _, off, size = sec(i)
        key = elf[stroff + name:elf.index(b"\0", stroff + name)].decode(errors="replace")
        out[key] = b"" if typ == 8 else elf[off:off + size]
    return out


_BUNDLE_MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def _device_code(fatbin: bytes):
    """The machine-code sections (.text, .rodata kernel descriptors, .note kernel metadata) of
    every amdgcn code object in a .hip_fatbin section, concatenated in bundle order; or None
    when the section holds no parsable offload bundle."""
    import struct
    parts, pos = [], fatbin.find(_BUNDLE_MAGIC)
    while pos >= 0:
        n, = struct.unpack_from("<Q", fatbin, pos + 24)
        cur = pos + 32
        for _ in range(n):
            off, size, tlen = struct.unpack_from("<QQQ", fatbin, cur)
            triple = fatbin[cur + 24:cur + 24 + tlen]
            cur += 24 + tlen
            if b"amdgcn" in triple and size:
                secs = _elf_sections(fatbin[pos + off:pos + off + size])
                parts += [triple] + [secs.get(k, b"") for k in (".text", ".rodata", ".note")]
        pos = fatbin.find(_BUNDLE_MAGIC, cur)
    return b"".join(parts) if parts else None


def code_object_id(path: str = LIB_PATH) -> str:
    """Identity of the device code in libnttmul.so: sha256 (16 hex digits) of the machine code of
    its gfx950 code objects -- each one's .text, .rodata (kernel descriptors) and .note (kernel
    metadata: names, register and LDS counts) -- read from the .hip_fatbin section's offload
    bundles (the whole section when it holds none).  Symbol tables are left out: they carry
    the compiler's per-source `__hip_cuid_*` marker, which changes with any edit of the .hip
    file even when no kernel does.  Host-only changes keep the id; any kernel change alters it.
    bench.py keys the committed PMC/ISA profiles (profiles/) by it, so a profile of another
    build is never reported as this build's."""
    import hashlib
    with open(path, "rb") as f:
        elf = f.read()
    if elf[:4] != b"\x7fELF" or elf[4] != 2:
        raise ValueError(f"{path}: not an ELF64 file")
    fat = _elf_sections(elf).get(".hip_fatbin")
    if fat is None:
        raise ValueError(f"{path}: no .hip_fatbin section")
    code = _device_code(fat)
    return hashlib.sha256(fat if code is None else code).hexdigest()[:16]


def _amdgcn_elfs(path: str) -> list:
    """The gfx950 code objects (ELF images) of a HIP shared library's .hip_fatbin offload bundles."""
    import struct
    with open(path, "rb") as f:
        elf = f.read()
    fat = _elf_sections(elf).get(".hip_fatbin")
    if fat is None:
        raise ValueError(f"{path}: no .hip_fatbin section")
    out, pos = [], fat.find(_BUNDLE_MAGIC)
    while pos >= 0:
        n, = struct.unpack_from("<Q", fat, pos + 24)
        cur = pos + 32
        for _ in range(n):
            off, size, tlen = struct.unpack_from("<QQQ", fat, cur)
            triple = fat[cur + 24:cur + 24 + tlen]
            cur += 24 + tlen
            if b"amdgcn" in triple and size:
                out.append(fat[pos + off:pos + off + size])
        pos = fat.find(_BUNDLE_MAGIC, cur)
    return out


def _elf_symbols(elf: bytes):
    """(name, value, size, type, section index) of every .symtab entry of an ELF64 image, and the
    (address, file offset) of each section."""
    import struct
    shoff, = struct.unpack_from("<Q", elf, 0x28)
    shentsize, shnum, _ = struct.unpack_from("<HHH", elf, 0x3A)
    secs = [struct.unpack_from("<IIQQQQIIQQ", elf, shoff + i * shentsize) for i in range(shnum)]
    syms = []
    for s in secs:
        if s[1] != 2:  # SHT_SYMTAB
            continue
        stroff = secs[s[6]][4]
        for k in range(s[5] // 24):
            name, info, _, shndx, value, size = struct.unpack_from("<IBBHQQ", elf, s[4] + 24 * k)
            nm = elf[stroff + name:elf.index(b"\0", stroff + name)].decode(errors="replace")
            syms.append((nm, value, size, info & 15, shndx))
    return syms, [(s[3], s[4]) for s in secs]


_BUILTIN = {"j": "u32", "m": "u64", "y": "u64", "i": "i32", "l": "i64", "b": "bool", "h": "u8"}


def _demangle_args(s: str, i: int):
    """Template arguments I...E of an Itanium-mangled nttmul kernel name from position i (at the
    'I'), as short strings ("Arith32P3", "u32", "12", "false"); returns (args, next position) or
    None for a form the kernels do not use."""
    assert s[i] == "I"
    i += 1
    args = []
    while s[i] != "E":
        c = s[i]
        if c in _BUILTIN:
            args.append(_BUILTIN[c])
            i += 1
        elif c == "L":  # literal: L<type><value>E, n = negative
            j = s.index("E", i)
            t, v = s[i + 1], s[i + 2:j]
            v = "-" + v[1:] if v.startswith("n") else v
            args.append({"0": "false", "1": "true"}[v] if t == "b" else v)
            i = j + 1
        elif s.startswith("NS_", i):  # nttmul::<id>[<args>]
            i += 3
            j = i
            while s[j].isdigit():
                j += 1
            ln = int(s[i:j])
            name = s[j:j + ln]
            i = j + ln
            if s[i] == "I":
                sub = _demangle_args(s, i)
                if sub is None:
                    return None
                name += "<" + ",".join(sub[0]) + ">"
                i = sub[1]
            if s[i] != "E":
                return None
            i += 1
            args.append(name)
        else:
            return None
    return args, i + 1


def kernel_key(symbol: str) -> str:
    """Short name of a kernel symbol of libnttmul.so, e.g.
    _ZN6nttmul6k_rowsINS_9Arith32P3EjjLi12ELi0ELb0EEEv... -> k_rows<Arith32P3,u32,u32,12,0,false>
    (the mangled symbol itself for a form this small demangler does not cover)."""
    if not symbol.startswith("_ZN6nttmul"):
        return symbol
    i = len("_ZN6nttmul")
    j = i
    while j < len(symbol) and symbol[j].isdigit():
        j += 1
    if j == i:
        return symbol
    ln = int(symbol[i:j])
    name = symbol[j:j + ln]
    k = j + ln
    if k < len(symbol) and symbol[k] == "I":
        try:
            r = _demangle_args(symbol, k)
        except (IndexError, KeyError, ValueError):
            r = None
        if r is None:
            return symbol
        return name + "<" + ",".join(r[0]) + ">"
    return name


def dispatch_key(name: str) -> str:
    """The kernel_key of one kernel named the way the library's dispatch describes it
    (nttmul_kernel_name: "k_rows<Arith32P3,u32,u32,12,0>", "...,prio>", "k_cols8<Arith64,u64,fwd>",
    "k_cols_fwd<Arith64,u64,4>"): the template arguments the short names leave out are filled in
    as kernels.hip instantiates them."""
    import re
    m = re.fullmatch(r"(\w+)<(.*)>", name.strip())
    if not m:
        return name.strip()
    kern, args = m.group(1), m.group(2).split(",")
    if kern == "k_rows":
        prio = args[-1] == "prio"
        args = (args[:-1] if prio else args) + ["true" if prio else "false"]
    elif kern == "k_cols_fwd":
        args = args + ["2"]
    elif kern == "k_cols8":
        w = "u64" if args[0] == "Arith64" else "u32"
        args = ([args[0], args[1], w, "0", "2"] if args[2] == "fwd" else [args[0], w, args[1], "1", "1"])
    return f"{kern}<{','.join(args)}>"


def kernel_hashes(path: str = LIB_PATH) -> dict:
    """Identity of every kernel in libnttmul.so's gfx950 code object, one by one: {kernel_key:
    sha256 (16 hex digits) of the kernel's machine code (its .text range) and its 64-byte kernel
    descriptor (<symbol>.kd: register, LDS, scratch and kernarg sizes), with the descriptor's
    kernel_code_entry_byte_offset (bytes 16-23, the distance from descriptor to code, which moves
    with every other kernel's size) zeroed}.  The kernels take everything through their arguments
    (no PC-relative data: no s_getpc_b64 in the listing), so a kernel's bytes change only when
    its own code does: a profile keyed by these hashes stays valid across edits of other kernels
    and of host code, and a claim "kernel X unchanged" is checkable (code_object_id is the
    whole-object digest)."""
    import hashlib
    out = {}
    for co in _amdgcn_elfs(path):
        syms, secs = _elf_symbols(co)
        by_name = {s[0]: s for s in syms}
        for nm, value, size, typ, shndx in syms:
            if typ != 2 or not size or nm + ".kd" not in by_name:  # STT_FUNC with a descriptor
                continue
            addr, off = secs[shndx]
            code = co[off + value - addr:off + value - addr + size]
            kd = by_name[nm + ".kd"]
            kaddr, koff = secs[kd[4]]
            desc = bytearray(co[koff + kd[1] - kaddr:koff + kd[1] - kaddr + 64])
            desc[16:24] = bytes(8)
            out[kernel_key(nm)] = hashlib.sha256(code + bytes(desc)).hexdigest()[:16]
    return out


def dispatched_kernel_hashes(names: str, path: str = LIB_PATH) -> dict:
    """{kernel_key: kernel hash}, in dispatch order, for a nttmul_kernel_name string
    ("a + b + c"); raises KeyError naming a kernel the code object does not hold."""
    table = kernel_hashes(path)
    out = {}
    for nm in (x.strip() for x in names.split("+")):
        key = dispatch_key(nm)
        if key not in table:
            raise KeyError(f"{nm} ({key}) is not a kernel of {path}")
        out[key] = table[key]
    return out


def exported_symbols() -> list:
    """Function names declared in include/nttmul.h (for the ABI completeness test)."""
    import re
    text = open(HEADER_PATH).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?(?:int|void|char\s*\*|const char \*)\s*\*?\s*"
                                 r"(nttmul_\w+|i?ntt256_\w+|ntt_red256_\w+|mulntt256_\w+|"
                                 r"inttmul256_\w+)\s*\(", text, re.M)))


def strerror(status: int) -> str:
    return load_library().nttmul_strerror(status).decode()


def _ptr(x) -> int:
    """Raw address of a numpy array or a torch tensor (device pointer for CUDA/HIP tensors)."""
    if isinstance(x, np.ndarray):
        assert x.flags.c_contiguous
        return x.ctypes.data
    if hasattr(x, "data_ptr"):
        assert x.is_contiguous()
        return x.data_ptr()
    return int(x)


def _dev_arg(x, batch: int, n: int, word_bits: int, dev: int) -> int:
    """Device pointer of an operand of a *_device call, after checking what the C ABI cannot:
    a torch tensor must hold at least batch * n words of word_bits on HIP device `dev`
    (a raw integer address is passed through unchecked, as in C)."""
    if word_bits not in (32, 64):
        raise ValueError("word_bits must be 32 or 64")
    if hasattr(x, "data_ptr"):
        if not x.is_contiguous():
            raise ValueError("device operands must be contiguous")
        if x.element_size() * 8 != word_bits:
            raise ValueError(f"tensor of {x.element_size() * 8}-bit elements for word_bits={word_bits}")
        if x.numel() < batch * n:
            raise ValueError(f"tensor of {x.numel()} words < batch * n = {batch * n}")
        if x.device.type != "cuda" or x.device.index != dev:
            raise ValueError(f"tensor on {x.device}, context call on device {dev}")
        return x.data_ptr()
    return _ptr(x)


class Context:
    """An (n, q) multiplier bound to one or more HIP devices (≙ an opened FPGA handle)."""

    def __init__(self, n: int, q: int, psi: int = 0, ndev: int = 1, first_dev: int = 0,
                 validate: bool = False, cyclic: bool = False, share_devices: bool = False,
                 issue_prio: int = 0, zero_copy_kb: int = 0, copy_threads: int = 0,
                 scratch_mb: int = 0, small_server: int = 0,
                 _lib: Optional[ctypes.CDLL] = None):
        """cyclic=True: FPGA-compat product mod (x^n - 1, q) (Hardware_Multiplier/PolyMult.v);
        `psi` then carries the primitive n-th root omega (0 = the smallest one).
        share_devices=True: `ndev` slices may map several onto one device (round-robin).
        issue_prio, zero_copy_kb, copy_threads, scratch_mb, small_server: the nttmul_params
        dispatch knobs (include/nttmul.h; 0 = the library default)."""
        self._lib = load_library() if _lib is None else _lib
        self._h = ctypes.c_void_p()
        flags = ((NTTMUL_FLAG_VALIDATE if validate else 0) | (NTTMUL_FLAG_CYCLIC if cyclic else 0)
                 | (NTTMUL_FLAG_SHARE_DEVICES if share_devices else 0))
        prm = _Params(n, q, psi, ndev, first_dev, flags, issue_prio, zero_copy_kb, copy_threads,
                      scratch_mb, small_server)
        st = self._lib.nttmul_create_sized(ctypes.byref(self._h), ctypes.byref(prm),
                                           ctypes.sizeof(prm))
        if st != NTTMUL_OK:
            raise NttmulError(st, strerror(st))
        info = Info()
        self._lib.nttmul_get_info(self._h, ctypes.byref(info))
        self.info = info
        self.n, self.q, self.psi = info.n, info.q, info.psi
        self.word_bits = info.word_bits
        self.first_dev = first_dev

    def close(self):
        if getattr(self, "_h", None) and self._h.value:
            self._lib.nttmul_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def _check(self, st: int):
        if st != NTTMUL_OK:
            raise NttmulError(st, f"{strerror(st)}: {self._lib.nttmul_last_error(self._h).decode()}")

    def last_host_path(self) -> int:
        """nttmul_last_host_path: 0 staged, 1 direct DMA, 2 zero-copy, 3 device server, -1 no
        call yet."""
        return int(self._lib.nttmul_last_host_path(self._h))

    def server_status(self):
        """nttmul_server_status: (setup / launch failures of the device server so far, the last
        one's message)."""
        buf = ctypes.create_string_buffer(256)
        n = self._lib.nttmul_server_status(self._h, buf, len(buf))
        if n < 0:
            self._check(n)
        return int(n), buf.value.decode()

    def kernel_name(self, word_bits: int = 0, batch: int = 0) -> str:
        """The device kernel(s) a product call of `batch` polynomials dispatches to
        (nttmul_kernel_name_batch; batch 0 = a large batch), e.g. "k_rows<Arith32P3,u32,u32,12,0>",
        or "k_rows<Arith32P,u32,u32,10,0,prio>" for a batch of at most 4 waves per SIMD."""
        word_bits = word_bits or (32 if self.q < (1 << 32) else 64)
        buf = ctypes.create_string_buffer(256)
        st = self._lib.nttmul_kernel_name_batch(self._h, word_bits, batch, buf, len(buf))
        if st < 0:
            self._check(st)
        return buf.value.decode()

    def last_kernel_name(self) -> str:
        """The kernel(s) the last product call launched (nttmul_last_kernel_name; "" before)."""
        buf = ctypes.create_string_buffer(256)
        st = self._lib.nttmul_last_kernel_name(self._h, buf, len(buf))
        if st < 0:
            self._check(st)
        return buf.value.decode()

    @property
    def io_dtype(self):
        return np.uint32 if self.q < (1 << 32) else np.uint64

    def multiply(self, a, b, dtype=None, out=None) -> np.ndarray:
        """c = a * b mod (x^n + 1, q) for host arrays of shape [n] or [batch, n].  `out`: the
        result array (same shape and dtype); with a, b and out in page-locked memory
        (host_empty) the library DMAs straight from and to them instead of staging."""
        dtype = dtype or self.io_dtype
        a = np.ascontiguousarray(a, dtype=dtype)
        b = np.ascontiguousarray(b, dtype=dtype)
        if a.shape != b.shape or a.shape[-1] != self.n:
            raise ValueError("a and b must both have shape [..., n]")
        if out is not None and (out.shape != a.shape or out.dtype != a.dtype
                                or not out.flags.c_contiguous):
            raise ValueError("out must be a C-contiguous array of a's shape and dtype")
        c = np.empty_like(a) if out is None else out
        batch = a.size // self.n
        fn = self._lib.nttmul_multiply_batch_u32 if dtype == np.uint32 else self._lib.nttmul_multiply_batch_u64
        self._check(fn(self._h, c.ctypes.data, a.ctypes.data, b.ctypes.data, batch))
        return c

    def _unary(self, op: str, x, dtype=None) -> np.ndarray:
        dtype = dtype or self.io_dtype
        x = np.ascontiguousarray(x, dtype=dtype)
        if x.shape[-1] != self.n:
            raise ValueError("input must have shape [..., n]")
        out = np.empty_like(x)
        w = "u32" if dtype == np.uint32 else "u64"
        fn = getattr(self._lib, f"nttmul_{op}_batch_{w}")
        self._check(fn(self._h, out.ctypes.data, x.ctypes.data, x.size // self.n))
        return out

    def forward(self, a, dtype=None) -> np.ndarray:
        """Negacyclic forward NTT, bit-reversed output (NTT/ntt.C:342 mulntt_ct_std2rev)."""
        return self._unary("forward", a, dtype)

    def inverse(self, a_hat, dtype=None) -> np.ndarray:
        """Inverse of forward(): nttmul_gs_rev2std (NTT/ntt.C:428) then n^-1."""
        return self._unary("inverse", a_hat, dtype)

    def transform(self, x, mode: int, dtype=None) -> np.ndarray:
        """nttmul_transform_batch: mode = XF_FORWARD/XF_INVERSE | XF_STD2REV/XF_REV2STD
        [| XF_UNSCALED] — the reference's wrapper set (NTT/ntt256.h:20-69) for this context."""
        dtype = dtype or self.io_dtype
        x = np.ascontiguousarray(x, dtype=dtype)
        if x.shape[-1] != self.n:
            raise ValueError("input must have shape [..., n]")
        out = np.empty_like(x)
        w = "u32" if dtype == np.uint32 else "u64"
        fn = getattr(self._lib, f"nttmul_transform_batch_{w}")
        self._check(fn(self._h, mode, out.ctypes.data, x.ctypes.data, x.size // self.n))
        return out

    def transform_device(self, out, x, mode: int, batch: int, word_bits: int,
                         dev: Optional[int] = None, stream: int = 0):
        dev = self.first_dev if dev is None else dev
        args = [_dev_arg(t, batch, self.n, word_bits, dev) for t in (out, x)]
        self._check(self._lib.nttmul_transform_device(self._h, mode, *args, batch,
                                                      word_bits, dev, stream or None))

    def pointwise(self, a, b, dtype=None) -> np.ndarray:
        """c[i] = a[i] * b[i] mod q (NTT/ntt.C:131 mul_array)."""
        dtype = dtype or self.io_dtype
        a = np.ascontiguousarray(a, dtype=dtype)
        b = np.ascontiguousarray(b, dtype=dtype)
        if a.shape != b.shape or a.shape[-1] != self.n:
            raise ValueError("a and b must both have shape [..., n]")
        c = np.empty_like(a)
        w = "u32" if dtype == np.uint32 else "u64"
        fn = getattr(self._lib, f"nttmul_pointwise_batch_{w}")
        self._check(fn(self._h, c.ctypes.data, a.ctypes.data, b.ctypes.data, a.size // self.n))
        return c

    def forward_device(self, out, a, batch: int, word_bits: int, dev: Optional[int] = None,
                       stream: int = 0):
        dev = self.first_dev if dev is None else dev
        args = [_dev_arg(t, batch, self.n, word_bits, dev) for t in (out, a)]
        self._check(self._lib.nttmul_forward_batch_device(self._h, *args, batch,
                                                          word_bits, dev, stream or None))

    def inverse_device(self, out, a, batch: int, word_bits: int, dev: Optional[int] = None,
                       stream: int = 0):
        dev = self.first_dev if dev is None else dev
        args = [_dev_arg(t, batch, self.n, word_bits, dev) for t in (out, a)]
        self._check(self._lib.nttmul_inverse_batch_device(self._h, *args, batch,
                                                          word_bits, dev, stream or None))

    def pointwise_device(self, c, a, b, batch: int, word_bits: int, dev: Optional[int] = None,
                         stream: int = 0):
        dev = self.first_dev if dev is None else dev
        args = [_dev_arg(t, batch, self.n, word_bits, dev) for t in (c, a, b)]
        self._check(self._lib.nttmul_pointwise_batch_device(self._h, *args,
                                                            batch, word_bits, dev, stream or None))

    def multiply_device(self, c, a, b, batch: int, word_bits: int, dev: Optional[int] = None,
                        stream: int = 0):
        """Device-resident batch (pointers or torch tensors on `dev`), enqueued on `stream`."""
        dev = self.first_dev if dev is None else dev
        args = [_dev_arg(t, batch, self.n, word_bits, dev) for t in (c, a, b)]
        self._check(self._lib.nttmul_multiply_batch_device(self._h, *args, batch,
                                                           word_bits, dev, stream or None))

    def fill_random_device(self, a, b, p0: int, count: int, word_bits: int, seed: int = SEED,
                           dev: Optional[int] = None, stream: int = 0):
        dev = self.first_dev if dev is None else dev
        args = [_dev_arg(t, count, self.n, word_bits, dev) for t in (a, b)]
        self._check(self._lib.nttmul_fill_random_device(self._h, *args, p0, count, seed,
                                                        word_bits, dev, stream or None))


# ---- planner API ------------------------------------------------------------

class _HostBlock:
    """Owner of one nttmul_host_alloc block (freed with the last numpy view of it)."""

    def __init__(self, nbytes: int):
        lib = load_library()
        lib.nttmul_host_alloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
        lib.nttmul_host_free.argtypes = [ctypes.c_void_p]
        lib.nttmul_host_free.restype = None
        p = ctypes.c_void_p()
        st = lib.nttmul_host_alloc(ctypes.byref(p), nbytes)
        if st != NTTMUL_OK:
            raise NttmulError(st, strerror(st))
        self._lib, self.ptr, self.nbytes = lib, p.value, nbytes

    def __del__(self):
        if getattr(self, "ptr", None):
            self._lib.nttmul_host_free(self.ptr)
            self.ptr = None


def host_empty(shape, dtype) -> np.ndarray:
    """Uninitialised numpy array in page-locked host memory (nttmul_host_alloc): host-buffer
    calls whose operands all live in such arrays DMA directly, without the staging copy."""
    dtype = np.dtype(dtype)
    count = int(np.prod(shape))
    blk = _HostBlock(max(1, count * dtype.itemsize))
    buf = (ctypes.c_char * blk.nbytes).from_address(blk.ptr)
    buf._nttmul_block = blk                      # the ctypes buffer keeps the block alive
    return np.frombuffer(buf, dtype=dtype, count=count).reshape(shape)


def is_prime(q: int) -> bool:
    return bool(load_library().nttmul_is_prime(q))


def smallest_psi(n: int, q: int) -> int:
    """generate_params.C:25-44: smallest element of order exactly 2n (0 if none)."""
    return int(load_library().nttmul_smallest_psi(n, q))


def smallest_omega(n: int, q: int) -> int:
    return int(load_library().nttmul_smallest_omega(n, q))


def find_prime(n: int, bits: int, cyclic: bool = False) -> int:
    """Largest prime q < 2^bits with q == 1 (mod 2n) (mod n if cyclic)."""
    q = ctypes.c_uint64()
    st = load_library().nttmul_find_prime(n, bits, int(cyclic), ctypes.byref(q))
    if st != NTTMUL_OK:
        raise NttmulError(st, strerror(st))
    return q.value


def table(n: int, q: int, name: str, psi: int = 0) -> np.ndarray:
    """One of the NTT/ntt.h:63-183 tables for (n, q, psi)."""
    out = np.zeros(n, dtype=np.uint64)
    st = load_library().nttmul_table(n, q, psi, TABLES.index(name), out.ctypes.data)
    if st != NTTMUL_OK:
        raise NttmulError(st, strerror(st))
    return out


def fpga_R(n: int, K: int) -> int:
    return int(load_library().nttmul_fpga_R(n, K))


def fpga_twiddles(n: int, q: int, w: int, R: int, P: int = 8) -> np.ndarray:
    """generate_twiddles (generate_params.C:54-73): the PolyMult.v W / W_INV stream."""
    lib = load_library()
    cnt = lib.nttmul_fpga_twiddles(n, q, w, R, P, None, 0)
    out = np.zeros(cnt, dtype=np.uint64)
    lib.nttmul_fpga_twiddles(n, q, w, R, P, out.ctypes.data, cnt)
    return out


# ---- text formats ------------------------------------------------------------

def read_coefficients(path: str, max_count: int) -> np.ndarray:
    """time_testing256.c:17-44 ler_coeficientes."""
    out = np.zeros(max_count, dtype=np.int32)
    cnt = load_library().nttmul_read_coefficients(path.encode(), out.ctypes.data, max_count)
    if cnt < 0:
        raise OSError(f"cannot open {path}")
    return out[:cnt]


def read_hex(path: str, max_count: int) -> np.ndarray:
    out = np.zeros(max_count, dtype=np.uint64)
    cnt = load_library().nttmul_read_hex(path.encode(), out.ctypes.data, max_count)
    if cnt < 0:
        raise OSError(f"cannot open {path}")
    return out[:cnt]


def write_hex(path: str, a) -> None:
    a = np.ascontiguousarray(a, dtype=np.uint64)
    if load_library().nttmul_write_hex(path.encode(), a.ctypes.data, a.size) < 0:
        raise OSError(f"cannot write {path}")


def multiply(a, b, n: int, q: int) -> np.ndarray:
    """multiply(a, b, n, q) -> c: the north-star entry point, one-shot."""
    with Context(n, q) as ctx:
        return ctx.multiply(a, b)


def _product256(name: str, c: np.ndarray, a: np.ndarray, b: np.ndarray) -> None:
    for x in (a, b, c):
        if not (isinstance(x, np.ndarray) and x.dtype == np.int32 and x.size == 256
                and x.flags.c_contiguous):
            raise TypeError("ntt256 products take contiguous int32 arrays of 256 coefficients")
    getattr(load_library(), name)(c.ctypes.data, a.ctypes.data, b.ctypes.data)


def ntt256_product1(c: np.ndarray, a: np.ndarray, b: np.ndarray) -> None:
    """NTT/ntt256.C:5 — c = a * b at n = 256, q = 12289 (result written into c)."""
    _product256("ntt256_product1", c, a, b)


def ntt256_product4(c: np.ndarray, a: np.ndarray, b: np.ndarray) -> None:
    """NTT/ntt256.C:16."""
    _product256("ntt256_product4", c, a, b)


def ntt_red256_product1(c: np.ndarray, a: np.ndarray, b: np.ndarray) -> None:
    """NTT-RED/ntt_red256.C:5."""
    _product256("ntt_red256_product1", c, a, b)


def ntt_red256_product4(c: np.ndarray, a: np.ndarray, b: np.ndarray) -> None:
    """NTT-RED/ntt_red256.C:30."""
    _product256("ntt_red256_product4", c, a, b)


def ntt256_transform(name: str, a: np.ndarray) -> None:
    """One of the reference's n = 256 wrappers (NTT/ntt256.h:20-69, e.g. "ntt256_ct_std2rev",
    "inttmul256_gs_rev2std") in place on a contiguous int32 array of 256 coefficients."""
    if name not in NTT256_WRAPPERS:
        raise ValueError(f"unknown ntt256 wrapper {name}")
    if not (isinstance(a, np.ndarray) and a.dtype == np.int32 and a.size == 256
            and a.flags.c_contiguous):
        raise TypeError("ntt256 wrappers take a contiguous int32 array of 256 coefficients")
    getattr(load_library(), name)(a.ctypes.data)

"""ctypes binding of libmvml_gat.so (the C ABI declared in include/mvml_gat.h).

The argument types of every entry point are parsed from the header itself, so the binding
cannot drift from the ABI.  There is deliberately no fallback: if the shared library is
missing or fails to load, every op raises.
"""
import collections
import ctypes
import os
import re

import torch  # noqa: F401  (import first: the library then binds torch's HIP runtime)

_PKG = os.path.dirname(os.path.abspath(__file__))
_DEFAULT_LIB = os.path.join(_PKG, "libmvml_gat.so")
LIB_PATH = os.environ.get("MVML_GAT_LIB", _DEFAULT_LIB)
HEADER_PATH = os.path.normpath(os.path.join(_PKG, "..", "..", "include", "mvml_gat.h"))

_CTYPE = {
    "int64_t": ctypes.c_int64,
    "int": ctypes.c_int,
    "uint32_t": ctypes.c_uint32,
    "float": ctypes.c_float,
    "double": ctypes.c_double,
    "size_t": ctypes.c_size_t,
    "void": None,
}


def _strip_comments(text):
    text = re.sub(r"/\*.*?\*/", " ", text, flags=re.S)
    text = re.sub(r"//[^\n]*", " ", text)
    return re.sub(r"^\s*#[^\n]*", " ", text, flags=re.M)  # preprocessor lines


def parse_header(path=HEADER_PATH):
    """Return {name: (restype, [argtypes])} for every mvml_* prototype in the header."""
    with open(path) as f:
        text = _strip_comments(f.read())
    protos = {}
    for m in re.finditer(r"([A-Za-z_][\w\s\*]*?)\b(mvml_\w+)\s*\(([^)]*)\)\s*;", text):
        ret, name, args = m.group(1).strip(), m.group(2), m.group(3).strip()
        protos[name] = (_ctype_of(ret, is_ret=True), [_ctype_of(a) for a in _split_args(args)])
    return protos


def _split_args(args):
    if args in ("", "void"):
        return []
    return [a.strip() for a in args.split(",")]


def _ctype_of(decl, is_ret=False):
    if "*" in decl:
        if is_ret and "char" in decl:
            return ctypes.c_char_p
        return ctypes.c_void_p
    toks = [t for t in decl.replace("const", " ").split() if t]
    base = toks[0]
    if base not in _CTYPE:
        raise ValueError(f"unsupported type in header: {decl!r}")
    return _CTYPE[base]


class MvmlError(RuntimeError):
    pass


_lib = None
_protos = None


def lib():
    """Load (once) and return the ctypes library with argtypes set from the header."""
    global _lib, _protos
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise MvmlError(
            f"libmvml_gat.so not found at {LIB_PATH}: build it with "
            "`python mvml-mpi_amd/build.py` (or __graft_entry__.build()); there is no CPU fallback")
    handle = ctypes.CDLL(LIB_PATH)
    protos = parse_header()
    for name, (res, args) in protos.items():
        try:
            fn = getattr(handle, name)
        except AttributeError:
            # only an alternate build (MVML_GAT_LIB, A/B runs of an older library) may lack an
            # entry point; the in-tree library exports every one (tests/test_host_cpu.py)
            if LIB_PATH == _DEFAULT_LIB:
                raise
            continue
        fn.restype = res
        fn.argtypes = args
    _lib, _protos = handle, protos
    return _lib


def exported_symbols():
    lib()
    return sorted(_protos)


class KernelTimer:
    """Optional HIP-event bracketing of selected entry points on the launching stream (torch's
    current stream, which is where every call enqueues).  bench.py enables it over its timed
    region to measure per-kernel average durations live; disabled it costs one dict lookup."""

    def __init__(self):
        self.names = set()
        self.events = {}
        self.tags = {}

    def enable(self, names):
        self.names = set(names)
        self.events = {n: [] for n in names}

    def disable(self):
        self.names = set()

    def record(self, name, start, end, tag):
        self.events[name].append((start, end, tag))

    def summary(self):
        """{name: [(ms, tag), ...]} — synchronises."""
        torch.cuda.synchronize()
        return {n: [(s.elapsed_time(e), tag) for s, e, tag in ev] for n, ev in self.events.items()}


timer = KernelTimer()
call_tag = [None]  # set by callers to attach per-call metadata (e.g. bytes moved) to a timing


def call(name, *args):
    """Invoke an int-returning entry point; raise MvmlError with mvml_last_error() on failure."""
    fn = getattr(lib(), name)
    tag, call_tag[0] = call_tag[0], None
    if name in timer.names:
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        rc = fn(*args)
        e.record()
        timer.record(name, s, e, tag)
    else:
        rc = fn(*args)
    if rc != 0:
        msg = lib().mvml_last_error().decode(errors="replace")
        raise MvmlError(f"{name} failed (status {rc}): {msg}")


# Kernel-path options (include/mvml_gat.h MVML_OPT_*): tests and tools switch paths through the
# C ABI; the environment variables only seed the defaults when the library loads.
OPTIONS = {"big_window": 0, "bwd_atomwise": 1, "gemm_tile": 2, "gemm_persist": 3, "gemm_nsplit": 4,
           "gemm_ring": 5, "lstm_tile": 6, "mean_src": 7, "flat_src": 8, "dst_fwd": 9,
           "dst_unr": 10, "smallk": 11}


class option:
    """Context manager: ``with option("big_window", 0): ...`` sets a kernel-path option and
    restores the previous value on exit."""

    def __init__(self, name, value):
        self.opt, self.value = OPTIONS[name], int(value)

    def __enter__(self):
        self.prev = lib().mvml_set_option(self.opt, self.value)
        if self.prev < 0:
            raise MvmlError(f"unknown option {self.opt}")
        return self

    def __exit__(self, *exc):
        lib().mvml_set_option(self.opt, self.prev)
        return False


def ptr(t):
    """Raw device pointer of a tensor (None -> NULL)."""
    if t is None:
        return None
    return ctypes.c_void_p(t.data_ptr())


def stream_ptr(device=None):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


_ws = collections.OrderedDict()
WS_STREAMS = 8  # scratch buffers kept (least recently used streams' buffers are dropped)


def workspace(nbytes, device):
    """Scratch buffer of the calling stream: one per (device, stream), so entry points enqueued
    on different streams never share scratch (the header's re-entrancy contract), and calls on
    one stream reuse it in stream order.  Growing allocates on the current stream and drops the
    old buffer there too, so the caching allocator hands it out again only behind the work that
    was enqueued on that stream before it (its blocks serve only allocations on that stream).
    At most WS_STREAMS streams keep a buffer: a transient stream's scratch is dropped once
    WS_STREAMS other streams have used the library since, never kept for the process lifetime."""
    dev = torch.device(device)
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    key = (idx, torch.cuda.current_stream(idx).cuda_stream)
    buf = _ws.get(key)
    if buf is None or buf.numel() < nbytes:
        buf = torch.empty(max(int(nbytes), 256), dtype=torch.uint8, device=dev)
        _ws[key] = buf
    _ws.move_to_end(key)
    while len(_ws) > WS_STREAMS:
        _ws.popitem(last=False)
    return buf


def ws_ptr_size(nbytes, device):
    if nbytes == 0:
        return None, 0
    buf = workspace(nbytes, device)
    return ctypes.c_void_p(buf.data_ptr()), buf.numel()

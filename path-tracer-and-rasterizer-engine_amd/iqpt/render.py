"""Render-context binding: ``PathTracer`` owns one iqpt_ctx (one GPU, one owned pixel set)."""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from ._lib import Camera, PacketDesc, PixelSet, check


def pixel_set(width: int, height: int, x0: int = 0, x1: int | None = None, y0: int = 0, ystep: int = 1,
              nrows: int | None = None) -> PixelSet:
    x1 = width if x1 is None else x1
    if nrows is None:
        nrows = (height - y0 + ystep - 1) // ystep
    return PixelSet(x0, x1, y0, ystep, nrows)


class PathTracer:
    """The MI355X render context (iqpt_create .. iqpt_destroy). Raises IqptError on failure."""

    def __init__(self, width: int, height: int, pixels: PixelSet | None = None, seed: int = _lib.DEFAULT_SEED,
                 max_depth: int = _lib.DEFAULT_MAX_DEPTH, device: int = 0):
        self._lib = _lib.load()
        h = C.c_void_p()
        ps = C.byref(pixels) if pixels is not None else None
        check(self._lib.iqpt_create(device, width, height, ps, seed, max_depth, C.byref(h)), "iqpt_create")
        self._h = h
        self.width, self.height = width, height
        self.pixels = pixels if pixels is not None else pixel_set(width, height)
        n = C.c_uint64()
        check(self._lib.iqpt_num_pixels(self._h, C.byref(n)), "iqpt_num_pixels")
        self.npix = n.value

    def close(self):
        if getattr(self, "_h", None):
            self._lib.iqpt_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self):
        return self._h

    def set_camera(self, cam: Camera):
        check(self._lib.iqpt_set_camera(self._h, C.byref(cam)), "iqpt_set_camera")

    def upload_packet(self, pk: PacketDesc):
        check(self._lib.iqpt_upload_packet(self._h, C.byref(pk)), "iqpt_upload_packet")

    def render(self, spp: int):
        check(self._lib.iqpt_render(self._h, spp), "iqpt_render")

    def sync(self):
        check(self._lib.iqpt_sync(self._h), "iqpt_sync")

    def reset(self):
        check(self._lib.iqpt_reset(self._h), "iqpt_reset")

    def read(self) -> tuple[np.ndarray, np.ndarray]:
        """(lin [npix,4] float32, bgra [npix,4] uint8) in the owned set's compact order."""
        lin = np.empty((self.npix, 4), dtype=np.float32)
        bgra = np.empty((self.npix, 4), dtype=np.uint8)
        check(self._lib.iqpt_read(self._h, lin.ctypes.data_as(C.POINTER(C.c_float)),
                                  bgra.ctypes.data_as(C.POINTER(C.c_uint8))), "iqpt_read")
        return lin, bgra

    def read_rng(self) -> np.ndarray:
        st = np.empty((self.npix, 6), dtype=np.uint32)
        check(self._lib.iqpt_read_rng(self._h, st.ctypes.data_as(C.POINTER(C.c_uint32))), "iqpt_read_rng")
        return st

    def checkpoint_save(self, path) -> None:
        """Accumulator, frame, RNG states, frame counter and ray count to `path` (iqpt_checkpoint_save)."""
        check(self._lib.iqpt_checkpoint_save(self._h, str(path).encode()), "iqpt_checkpoint_save")

    def checkpoint_load(self, path) -> None:
        """Resume from a checkpoint of a context with the same frame, pixel set, seed and max_depth."""
        check(self._lib.iqpt_checkpoint_load(self._h, str(path).encode()), "iqpt_checkpoint_load")

    def copy_accum_device(self, dst_ptr: int, nbytes: int):
        check(self._lib.iqpt_copy_accum_device(self._h, C.c_void_p(dst_ptr), nbytes), "iqpt_copy_accum_device")

    def copy_frame_device(self, dst_ptr: int, nbytes: int):
        """BGRA8 frame (npix uint32, compact order) into a device buffer (iqpt_copy_frame_device)."""
        check(self._lib.iqpt_copy_frame_device(self._h, C.c_void_p(dst_ptr), nbytes), "iqpt_copy_frame_device")

    def copy_frame_device_async(self, dst_ptr: int, nbytes: int):
        """The BGRA8 frame into a device buffer, enqueued on the context's stream (no host sync;
        iqpt_copy_frame_device_async). Order other work against frame_stream_handle(), asked
        right before this call (overlapped launches keep overlapping across the copy)."""
        check(self._lib.iqpt_copy_frame_device_async(self._h, C.c_void_p(dst_ptr), nbytes),
              "iqpt_copy_frame_device_async")

    def stream_handle(self) -> int:
        """The context's hipStream_t (iqpt_stream), e.g. for torch.cuda.ExternalStream."""
        s = C.c_void_p()
        check(self._lib.iqpt_stream(self._h, C.byref(s)), "iqpt_stream")
        return int(s.value or 0)

    def frame_stream_handle(self) -> int:
        """The hipStream_t copy_frame_device_async enqueues on now (iqpt_frame_stream): the last
        render's stream while overlapped launches are in flight, else stream_handle()."""
        s = C.c_void_p()
        check(self._lib.iqpt_frame_stream(self._h, C.byref(s)), "iqpt_frame_stream")
        return int(s.value or 0)

    # ---- multi-GPU frame delivery over RCCL, inside libiqpt (iqpt_comm_*, iqpt_gather_*)

    def comm_init(self, rank: int, world: int, uid: bytes):
        """Join the ranks of one frame's cyclic row split (collective; this context must own rank's rows,
        dist.pixel_set_for_rank). `uid` from comm_unique_id() on one rank, shared out of band."""
        b = (C.c_uint8 * _lib.COMM_ID_BYTES).from_buffer_copy(bytes(uid))
        check(self._lib.iqpt_comm_init(self._h, rank, world, b, _lib.COMM_ID_BYTES), "iqpt_comm_init")
        self._comm_rank = rank

    def gather_frame_async(self, root: int, dst_ptr: int, nbytes: int):
        """Collective: the BGRA8 frame gathered to `root` and assembled there (W x H uint32 into dst_ptr, a
        device buffer; ignored on other ranks), stream-ordered behind the renders issued so far
        (iqpt_gather_frame_async). Order reads of dst on comm_stream_handle()."""
        check(self._lib.iqpt_gather_frame_async(self._h, root, C.c_void_p(dst_ptr or None), nbytes),
              "iqpt_gather_frame_async")

    def gather_accum(self, root: int, dst_ptr: int, nbytes: int):
        """Collective, synchronous: the float4 accumulators of the whole frame on `root` (device buffer)."""
        check(self._lib.iqpt_gather_accum(self._h, root, C.c_void_p(dst_ptr or None), nbytes), "iqpt_gather_accum")

    def gather_read(self, root: int, what: str = "both"):
        """Collective, synchronous (every rank calls it with the same `what`): on `root` the whole frame's
        (lin [W*H,4] float32, bgra [W*H,4] uint8), row-major, with None for a plane not asked for ("accum",
        "frame" or "both"; iqpt_gather_read_select). Every other rank gets None (not a tuple: its host buffers
        are not touched). The root is told apart by the rank given to comm_init(), which must come first: a
        communicator set up another way raises here, instead of a root passing no buffers."""
        sel = {"accum": _lib.GATHER_ACCUM, "frame": _lib.GATHER_FRAME,
               "both": _lib.GATHER_ACCUM | _lib.GATHER_FRAME}[what]
        rank = getattr(self, "_comm_rank", None)
        if rank is None:
            raise RuntimeError("gather_read: call comm_init() on this PathTracer first (its rank decides the root)")
        is_root = root == rank
        lin = (np.empty((self.width * self.height, 4), dtype=np.float32)
               if is_root and sel & _lib.GATHER_ACCUM else None)
        bgra = (np.empty((self.width * self.height, 4), dtype=np.uint8)
                if is_root and sel & _lib.GATHER_FRAME else None)
        check(self._lib.iqpt_gather_read_select(
            self._h, root, sel, lin.ctypes.data_as(C.POINTER(C.c_float)) if lin is not None else None,
            bgra.ctypes.data_as(C.POINTER(C.c_uint8)) if bgra is not None else None), "iqpt_gather_read_select")
        return (lin, bgra) if is_root else None

    def comm_time(self) -> tuple[float, int]:
        """(ms, gathers): the gathers' summed durations on the communicator stream since the last call."""
        ms = C.c_double()
        n = C.c_uint64()
        check(self._lib.iqpt_comm_time(self._h, C.byref(ms), C.byref(n)), "iqpt_comm_time")
        return ms.value, n.value

    def comm_stream_handle(self) -> int:
        """The communicator's hipStream_t (iqpt_comm_stream): the gathers and the root's assembly run on it."""
        s = C.c_void_p()
        check(self._lib.iqpt_comm_stream(self._h, C.byref(s)), "iqpt_comm_stream")
        return int(s.value or 0)

    def set_split(self, mode: int):
        """Sample-parallel launches: _lib.SPLIT_AUTO (default), SPLIT_OFF, SPLIT_ON or SPLIT_SPEC (iqpt_set_split;
        SPLIT_CHAIN and SPLIT_FAN are refused since round 6, their kernels archived)."""
        check(self._lib.iqpt_set_split(self._h, mode), "iqpt_set_split")

    def set_overlap(self, mode: int):
        """Overlapped launches on two streams: _lib.OVERLAP_AUTO (default) or OVERLAP_OFF (iqpt_set_overlap)."""
        check(self._lib.iqpt_set_overlap(self._h, mode), "iqpt_set_overlap")

    def launch_mode(self) -> str:
        """How the last launch ran: "plain", "split" (speculative runs + stitch), "split+fan" (with the anchored
        tiles in the fan kernel) or "spec", from iqpt_debug_split_info. Synchronises."""
        import ctypes as C
        self._lib.iqpt_debug_split_info.argtypes = [C.c_void_p, C.POINTER(C.c_ulonglong)]
        info = (C.c_ulonglong * 8)()
        check(self._lib.iqpt_debug_split_info(self._h, info), "iqpt_debug_split_info")
        return {1: "split", 5: "split+fan", 6: "spec"}.get(int(info[7]), "plain")

    def kernel_span(self) -> float:
        """First start to last end (ms) of the launches of the last kernel_time() call (iqpt_kernel_span)."""
        ms = C.c_double()
        check(self._lib.iqpt_kernel_span(self._h, C.byref(ms)), "iqpt_kernel_span")
        return ms.value

    def prepare(self):
        """Build the tile masks / queue order / split set now (iqpt_prepare; synchronises)."""
        check(self._lib.iqpt_prepare(self._h), "iqpt_prepare")

    def frames(self) -> int:
        f = C.c_uint64()
        check(self._lib.iqpt_frame_count(self._h, C.byref(f)), "iqpt_frame_count")
        return f.value

    def rays(self) -> int:
        r = C.c_uint64()
        check(self._lib.iqpt_rays_traced(self._h, C.byref(r)), "iqpt_rays_traced")
        return r.value

    def kernel_time(self) -> tuple[float, int]:
        ms = C.c_double()
        n = C.c_uint64()
        check(self._lib.iqpt_kernel_time(self._h, C.byref(ms), C.byref(n)), "iqpt_kernel_time")
        return ms.value, n.value


def comm_unique_id() -> bytes:
    """An RCCL unique id for comm_init (iqpt_comm_unique_id): made on one rank, shared with the others."""
    b = (C.c_uint8 * _lib.COMM_ID_BYTES)()
    check(_lib.load().iqpt_comm_unique_id(b, _lib.COMM_ID_BYTES), "iqpt_comm_unique_id")
    return bytes(b)


def kernel_name() -> str:
    return _lib.load().iqpt_kernel_name().decode()


def write_ppm(path: str, width: int, height: int, bgra: np.ndarray):
    b = np.ascontiguousarray(bgra, dtype=np.uint8)
    check(_lib.load().iqpt_write_ppm(str(path).encode(), width, height, b.ctypes.data_as(C.POINTER(C.c_uint8))),
          "iqpt_write_ppm")

"""Checkpoint files of the lit-llama path: a weights-only, memory-mapped reader for every
`torch.save`-style zip checkpoint (including the reference's `incremental_save` output) and a
streaming writer for the converters.

Reference: lit_llama/utils.py:200-376 (`lazy_load`: a custom unpickler that defers reading each
tensor) and 492-531 (`incremental_save`: tensors written into the zip as they are produced, the
pickle last, protocol 5). scripts/convert_hf_checkpoint.py:88 writes `lit-llama.pth` with it, and
generate.py:126 reads it back with `lazy_load`.

`torch.load(weights_only=True)` refuses that file: protocol 5 puts FRAME opcodes in the pickle,
which torch's weights-only unpickler does not take. `lazy_load` here reads it without executing
anything from the file: its unpickler resolves exactly four kinds of globals -- the tensor and
parameter rebuild functions (mapped to local functions that only view bytes), the typed-storage
classes (mapped to dtypes) and `collections.OrderedDict` -- and refuses every other global. Each
storage record of the zip (stored uncompressed, as torch writes them) is memory-mapped copy-on-write
and viewed in place, so a tensor's pages are read when the tensor is used (the reference's lazy
loading) and nothing is written back to the file.

`incremental_save` writes a checkpoint tensor by tensor (each storage record goes into the zip
when `store_early` is called and its memory can be dropped right after), then the pickle. The
pickle is protocol 2, so `torch.load(weights_only=True)` reads these files as well.
"""
from __future__ import annotations

import collections
import io
import mmap
import pickle
import struct
import zipfile
from pathlib import Path

import torch

# typed-storage class name (how torch pickles a storage's type) -> dtype
_STORAGE_DTYPES = {
    "DoubleStorage": torch.float64, "FloatStorage": torch.float32, "HalfStorage": torch.float16,
    "BFloat16Storage": torch.bfloat16, "LongStorage": torch.int64, "IntStorage": torch.int32,
    "ShortStorage": torch.int16, "CharStorage": torch.int8, "ByteStorage": torch.uint8,
    "BoolStorage": torch.bool, "ComplexFloatStorage": torch.complex64, "ComplexDoubleStorage": torch.complex128,
}
_DTYPE_STORAGE = {v: k for k, v in _STORAGE_DTYPES.items()}


class _StorageType:
    """What a pickled storage class resolves to: only its dtype."""

    def __init__(self, dtype):
        self.dtype = dtype


class _StorageRef:
    """A persistent id of the pickle: record key, dtype, element count."""

    def __init__(self, key: str, dtype, numel: int):
        self.key, self.dtype, self.numel = key, dtype, numel


class _Archive:
    """The zip's storage records, memory-mapped copy-on-write and viewed as 1-D tensors."""

    def __init__(self, path: Path):
        self.path = Path(path)
        self._f = open(self.path, "rb")
        size = self.path.stat().st_size
        self._mm = mmap.mmap(self._f.fileno(), 0, access=mmap.ACCESS_COPY) if size else None
        with zipfile.ZipFile(self.path) as zf:
            infos = zf.infolist()
            pkl = [i for i in infos if i.filename == "data.pkl" or i.filename.endswith("/data.pkl")]
            if len(pkl) != 1:
                raise ValueError(f"{self.path}: not a torch zip checkpoint (no single data.pkl record)")
            self.prefix = pkl[0].filename[: -len("data.pkl")]
            self.pickle_bytes = zf.read(pkl[0])
            self.records = {}
            for i in infos:
                if not i.filename.startswith(self.prefix + "data/"):
                    continue
                if i.compress_type != zipfile.ZIP_STORED:
                    raise ValueError(f"{self.path}: record {i.filename} is compressed")
                self.records[i.filename[len(self.prefix) + 5:]] = (self._data_offset(i), i.file_size)
        self._f.close()  # the map stays valid without the descriptor
        self._views = {}

    def _data_offset(self, info: zipfile.ZipInfo) -> int:
        # local file header: 30 bytes, then the name and the extra field (torch pads it to align data)
        self._f.seek(info.header_offset)
        hdr = self._f.read(30)
        if hdr[:4] != b"PK\x03\x04":
            raise ValueError(f"{self.path}: bad local header for {info.filename}")
        n, m = struct.unpack("<HH", hdr[26:30])
        return info.header_offset + 30 + n + m

    def storage(self, ref: _StorageRef) -> torch.Tensor:
        key = (ref.key, ref.dtype)
        if key not in self._views:
            if ref.key not in self.records:
                raise ValueError(f"{self.path}: missing storage record data/{ref.key}")
            off, nbytes = self.records[ref.key]
            need = ref.numel * torch.empty((), dtype=ref.dtype).element_size()
            if need > nbytes:
                raise ValueError(f"{self.path}: record data/{ref.key} holds {nbytes} bytes, {need} expected")
            if ref.numel == 0:
                t = torch.empty(0, dtype=ref.dtype)
            else:
                t = torch.frombuffer(self._mm, dtype=ref.dtype, count=ref.numel, offset=off)
            self._views[key] = t
        return self._views[key]


def _rebuild_tensor(storage, storage_offset, size, stride, requires_grad=False, backward_hooks=None,
                    metadata=None):
    t = storage.as_strided(tuple(size), tuple(stride), storage_offset)
    if requires_grad:
        t.requires_grad_(True)
    return t


def _rebuild_parameter(data, requires_grad, backward_hooks, *args):
    return torch.nn.Parameter(data, requires_grad)


class _WeightsUnpickler(pickle.Unpickler):
    def __init__(self, data: bytes, archive: _Archive):
        super().__init__(io.BytesIO(data))
        self.archive = archive

    def find_class(self, module, name):
        if module == "torch._utils" and name == "_rebuild_tensor_v2":
            return _rebuild_tensor
        if module == "torch._utils" and name == "_rebuild_parameter":
            return _rebuild_parameter
        if module == "collections" and name == "OrderedDict":
            return collections.OrderedDict
        if module == "torch" and name in _STORAGE_DTYPES:
            return _StorageType(_STORAGE_DTYPES[name])
        raise pickle.UnpicklingError(f"checkpoint refers to {module}.{name}: not a weights-only object, refused")

    def persistent_load(self, pid):
        if not (isinstance(pid, tuple) and len(pid) == 5 and pid[0] in ("storage", b"storage")):
            raise pickle.UnpicklingError(f"unexpected persistent id {pid!r}")
        _, stype, key, _location, numel = pid
        if not isinstance(stype, _StorageType):
            raise pickle.UnpicklingError(f"unexpected storage type {stype!r}")
        return self.archive.storage(_StorageRef(str(key), stype.dtype, int(numel)))


def read_checkpoint(path) -> dict:
    """The object pickled in a torch zip checkpoint (a state dict), every tensor a view into the
    memory-mapped file (pages read on use). Nothing in the file is executed."""
    ar = _Archive(Path(path))
    return _WeightsUnpickler(ar.pickle_bytes, ar).load()


class lazy_load:
    """reference lit_llama/utils.py:364-376: `with lazy_load(path) as sd:` gives the checkpoint's
    state dict with the tensors read on use; reads `torch.save` files and the reference's
    `incremental_save` files alike."""

    def __init__(self, fn):
        self.sd = read_checkpoint(fn)

    def __enter__(self):
        return self.sd

    def __exit__(self, exc_type, exc_val, exc_tb):
        self.sd = None


class _TensorRecord:
    """Pickles as the reference's tensor reduction: _rebuild_tensor_v2(storage, offset, size,
    stride, requires_grad, OrderedDict())."""

    def __init__(self, ref: _StorageRef, size, stride, offset=0):
        self.ref, self.size, self.stride, self.offset = ref, tuple(size), tuple(stride), offset

    def __reduce_ex__(self, protocol):
        return (torch._utils._rebuild_tensor_v2,
                (self.ref, self.offset, self.size, self.stride, False, collections.OrderedDict()))


class _RecordPickler(pickle.Pickler):
    def persistent_id(self, obj):
        if isinstance(obj, _StorageRef):
            return ("storage", getattr(torch, _DTYPE_STORAGE[obj.dtype]), obj.key, "cpu", obj.numel)
        return None


class incremental_save:
    """reference lit_llama/utils.py:492-531: `with incremental_save(path) as saver:`
    `sd[k] = saver.store_early(tensor)` writes the tensor's bytes into the zip at once (the caller
    may drop the tensor right after), `saver.save(sd)` writes the pickle; at most one converted
    tensor need be alive at a time and the output is the only file written."""

    def __init__(self, name):
        self.name = Path(name)
        self._w = torch._C.PyTorchFileWriter(str(self.name))
        self.has_saved = False
        self.next_key = 0

    def __enter__(self):
        return self

    def store_early(self, tensor: torch.Tensor) -> _TensorRecord:
        if not isinstance(tensor, torch.Tensor):
            raise TypeError(f"can only store tensors early, not {type(tensor)}")
        if self.has_saved:
            raise RuntimeError("have already saved")
        if tensor.dtype not in _DTYPE_STORAGE:
            raise TypeError(f"dtype {tensor.dtype} is not a checkpoint storage type")
        t = tensor.detach().to("cpu").contiguous()
        if t.storage_offset() != 0 or t.untyped_storage().nbytes() != t.numel() * t.element_size():
            t = t.clone()  # the record is the whole storage: a view into a larger one is copied out
        key = str(self.next_key)
        self.next_key += 1
        self._w.write_record(f"data/{key}", t.untyped_storage(), t.numel() * t.element_size())
        return _TensorRecord(_StorageRef(key, t.dtype, t.numel()), t.shape, t.stride())

    def save(self, obj) -> None:
        if self.has_saved:
            raise RuntimeError("have already saved")
        buf = io.BytesIO()
        _RecordPickler(buf, protocol=2).dump(obj)
        data = buf.getvalue()
        self._w.write_record("data.pkl", data, len(data))
        self.has_saved = True

    def __exit__(self, exc_type, exc_val, exc_tb):
        self._w.write_end_of_file()

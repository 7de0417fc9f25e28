"""Shared test helpers: typed random inputs with edge values, byte comparison
with pair-type padding masked, and the per-case reference order."""
import numpy as np

from mvapich2_amd.consts import TYPES

EDGE_F = [np.nan, -np.nan, 0.0, -0.0, np.inf, -np.inf, 1.0, -1.0]


def data_mask(type_name, count):
    """Bytes that carry data (pair padding excluded)."""
    handle, desc, size, ext = TYPES[type_name]
    m = np.ones(count * ext, dtype=bool)
    if type_name == "MPI_LONG_DOUBLE":  # x87: 10 value bytes in a 16-byte slot
        m = m.reshape(count, ext)
        m[:, 10:] = False
        return m.ravel()
    if size != ext:
        m = m.reshape(count, ext)
        if type_name == "MPI_SHORT_INT":
            m[:, 2:4] = False
        else:
            m[:, 12:] = False
        m = m.ravel()
    return m


def np_dtype(type_name):
    desc = TYPES[type_name][1]
    if desc == "f16":
        return np.dtype(np.longdouble)
    return np.dtype(desc)


def rand_typed(type_name, count, rng, edges=True, small=False, ties=False):
    """Seeded random operand of `count` elements (as a byte-backed numpy array).  ties: floating
    values drawn from {+-0, +-1, two NaN payloads}, so every element's MAX / MIN result depends on
    which operand is the accumulator (signed-zero ties keep inout, NaN against NaN keeps inout)."""
    dt = np_dtype(type_name)
    if ties and dt.kind == "f":
        pool = np.array([0.0, -0.0, 1.0, -1.0, np.nan, np.nan], dtype=dt)
        if dt.itemsize == 4:
            pool[4:] = np.array([0x7FC00011, 0xFFC00022], dtype=np.uint32).view(np.float32)
        else:
            pool[4:] = np.array([0x7FF8000000000011, 0xFFF8000000000022], dtype=np.uint64).view(np.float64)
        return pool[rng.integers(0, len(pool), count)]
    if type_name == "MPI_C_BOOL":  # _Bool objects hold only 0 / 1 (other bytes are UB in C)
        return rng.integers(0, 2, count).astype(dt)
    if dt.names:
        x = np.zeros(count, dtype=dt)
        vt = dt["value"]
        if vt.kind == "f":
            v = np.floor(rng.uniform(-8, 8, count)).astype(vt)  # ties on purpose
            if edges and count >= 8:
                v[:4] = [np.nan, -0.0, 0.0, np.nan]
        else:
            v = rng.integers(-5, 5, count).astype(vt)
        x["value"] = v
        lt = dt["loc"]
        x["loc"] = rng.integers(0, 8, count).astype(lt)
        return x
    if dt.kind == "c":
        re = rng.standard_normal(count)
        im = rng.standard_normal(count)
        x = (re + 1j * im).astype(dt)
        if edges and count >= 8:
            e = np.array([complex(np.inf, np.nan), complex(np.nan, np.inf), complex(np.nan, np.nan),
                          complex(0.0, -0.0), complex(np.inf, 0.0), complex(1e38, 1e38)], dtype=dt)
            x[:6] = e[rng.permutation(6)]
        return x
    if dt.kind == "f":
        x = rng.standard_normal(count).astype(dt)
        if small:
            x = np.floor(rng.uniform(-4, 4, count)).astype(dt)
        if edges and count >= len(EDGE_F):
            e = np.array(EDGE_F, dtype=dt)
            if dt.itemsize == 4:  # NaNs with distinct payloads / signs
                e[0] = np.array([0x7FC00011], dtype=np.uint32).view(np.float32)[0]
                e[1] = np.array([0xFFA00022], dtype=np.uint32).view(np.float32)[0]  # signalling
            x[: len(EDGE_F)] = e[rng.permutation(len(EDGE_F))]
            if dt.itemsize >= 4 and count > 12:
                x[8] = np.finfo(dt).tiny / 4  # denormal
                x[9] = -np.finfo(dt).tiny / 8
                x[10] = np.finfo(dt).max
                x[11] = -np.finfo(dt).max
        return x
    if dt.kind in "iu":
        info = np.iinfo(dt)
        if small:
            x = rng.integers(0, 3, count).astype(dt)
        else:
            x = rng.integers(info.min, info.max, count, endpoint=True, dtype=dt)
        if edges and count >= 4 and not small:
            x[:4] = [info.min, info.max, 0, 1 if info.min == 0 else -1]
        return x
    raise ValueError(type_name)


def as_bytes(a):
    return np.ascontiguousarray(a).view(np.uint8).ravel()


def assert_bytes_equal(got, want, type_name, count, what=""):
    m = data_mask(type_name, count)
    g = as_bytes(got)[m]
    w = as_bytes(want)[m]
    if not np.array_equal(g, w):
        bad = np.nonzero(g != w)[0]
        ext = TYPES[type_name][3]
        e = bad[0] // ext if len(bad) else -1
        raise AssertionError(f"{what} {type_name}: {len(bad)} bytes differ, first element {e}")

"""Disparity / image file formats of the reference (utils/file_io.py).

* PFM read / write, byte-compatible with utils/file_io.py:37-99 (rows stored bottom-up,
  negative scale = little-endian, `'%f'` scale line);
* KITTI disparity PNG: uint16 = round-down(disp * 256) (inference.py:197-204), read back / 256
  (file_io.py:102-105).  The reference writes it with skimage (absent here); the writer below
  is a self-contained 16-bit grayscale PNG encoder (zlib, 'Up' row filter); reading uses PIL
  like the reference.
* read_img / read_disp with the reference's dispatch (file_io.py:11-34).
"""
import re
import struct
import sys
import zlib

import numpy as np


def read_img(filename):
    """file_io.py:11-14: RGB float32 [H, W, 3] in [0, 255]."""
    from PIL import Image
    return np.array(Image.open(filename).convert('RGB')).astype(np.float32)


def read_disp(filename, subset=False):
    """file_io.py:17-31: [H, W] disparity from .pfm (negated for the Scene Flow subset), KITTI
    .png or .npy."""
    if filename.endswith('pfm'):
        disp = np.ascontiguousarray(read_pfm(filename)[0])
        return -disp if subset else disp
    if filename.endswith('png'):
        return read_kitti_disp(filename)
    if filename.endswith('npy'):
        return np.load(filename)
    raise Exception('Invalid disparity file format!')


def read_pfm(filename):
    """file_io.py:34-70 -> (data [H, W] or [H, W, 3] float32, scale)."""
    with open(filename, 'rb') as f:
        header = f.readline().rstrip().decode('ascii')
        if header not in ('PF', 'Pf'):
            raise Exception('Not a PFM file.')
        dims = re.match(r'^(\d+)\s(\d+)\s$', f.readline().decode('ascii'))
        if not dims:
            raise Exception('Malformed PFM header.')
        width, height = map(int, dims.groups())
        scale = float(f.readline().decode('ascii').rstrip())
        endian = '<' if scale < 0 else '>'
        data = np.frombuffer(f.read(), endian + 'f')
    shape = (height, width, 3) if header == 'PF' else (height, width)
    return np.flipud(data.reshape(shape)), abs(scale)


def write_pfm(filename, image, scale=1):
    """file_io.py:73-99 (same bytes: header, '%d %d', '%f' scale with the endianness sign, rows
    bottom-up in native byte order)."""
    if image.dtype.name != 'float32':
        raise Exception('Image dtype must be float32.')
    image = np.flipud(image)
    if image.ndim == 3 and image.shape[2] == 3:
        color = True
    elif image.ndim == 2 or (image.ndim == 3 and image.shape[2] == 1):
        color = False
    else:
        raise Exception('Image must have H x W x 3, H x W x 1 or H x W dimensions.')
    endian = image.dtype.byteorder
    if endian == '<' or (endian == '=' and sys.byteorder == 'little'):
        scale = -scale
    with open(filename, 'wb') as f:
        f.write(b'PF\n' if color else b'Pf\n')
        f.write(b'%d %d\n' % (image.shape[1], image.shape[0]))
        f.write(b'%f\n' % scale)
        image.tofile(f)


def read_kitti_disp(filename):
    """file_io.py:102-105: uint16 PNG / 256."""
    from PIL import Image
    return np.array(Image.open(filename)).astype(np.float32) / 256.


def _chunk(tag, payload):
    body = tag + payload
    return struct.pack('>I', len(payload)) + body + struct.pack('>I', zlib.crc32(body) & 0xffffffff)


def encode_png_u16(gray):
    """16-bit grayscale PNG bytes of a [H, W] uint16 array (non-interlaced; every scanline
    'Up'-filtered -- byte-wise difference to the row above -- which suits smooth disparities)."""
    gray = np.ascontiguousarray(gray, dtype='>u2')
    h, w = gray.shape
    rows = gray.view(np.uint8).reshape(h, 2 * w)
    up = rows.copy()
    up[1:] = rows[1:] - rows[:-1]  # uint8 wrap-around, as PNG defines it
    raw = np.empty((h, 2 * w + 1), np.uint8)
    raw[:, 0] = 2  # filter type Up (row 0: the row above is zero)
    raw[:, 1:] = up
    ihdr = struct.pack('>IIBBBBB', w, h, 16, 0, 0, 0, 0)
    return (b'\x89PNG\r\n\x1a\n' + _chunk(b'IHDR', ihdr)
            + _chunk(b'IDAT', zlib.compress(raw.tobytes(), 6)) + _chunk(b'IEND', b''))


def write_kitti_disp(filename, disp):
    """inference.py:197-204: (disp * 256).astype(uint16) as a 16-bit PNG."""
    with open(filename, 'wb') as f:
        f.write(encode_png_u16((np.asarray(disp, np.float32) * 256.).astype(np.uint16)))

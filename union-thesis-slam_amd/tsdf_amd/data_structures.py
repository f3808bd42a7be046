"""Value objects of the hash API, mirroring data_structures/{hash_entry,voxel}.py.

The reference's HashEntry carries (position, offset, voxel) and its Voxel (sdf, colour,
weight); HashTable.add_hash_entry / get_hash_entry trade in them.  Here they are plain value
holders: the voxel state itself lives in HBM and is read or written through the C-ABI.
The reference's 5-slot `Bucket` has no counterpart -- the block table replaces the chained
buckets.
"""
from __future__ import annotations

import numpy as np


class Voxel:
    """data_structures/voxel.py:6-17: sdf=1, colour=0 (packed B*65536+G*256+R), weight=0."""

    def __init__(self, sdf=1, color=0, weight=0):
        self._sdf = sdf
        self._color = color
        self._weight = weight

    def get_sdf(self):
        return self._sdf

    def get_color(self):
        return self._color

    def get_weight(self):
        return self._weight

    def __repr__(self):
        return f"Voxel(sdf={self._sdf}, color={self._color}, weight={self._weight})"


class HashEntry:
    """data_structures/hash_entry.py:6-45.  `offset` is (table slot, voxel-in-block) once the
    entry is stored (the reference's (bucket, slot) pair)."""

    def __init__(self, position, offset, voxel):
        self._position = position
        self._offset = offset
        self._voxel = voxel

    def set_offset(self, pointer):
        self._offset = pointer

    def get_position(self):
        return self._position

    def get_voxel(self):
        return self._voxel

    def is_empty_offset(self):
        return self._offset is None

    def get_offset(self):
        return None if self._offset is None else self._offset

    def equals(self, hash_entry):
        return np.array_equal(self._position, hash_entry.get_position())

    def match_position(self, position):
        return np.array_equal(self._position, position)

    def __repr__(self):
        return f"HashEntry(position={list(self._position)}, offset={self._offset}, voxel={self._voxel})"

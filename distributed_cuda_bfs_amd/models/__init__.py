"""BFS front-ends.  The "model family" of this framework is the set of
traversal algorithms the engine implements:

  ref     the reference algorithm (thread per frontier vertex, atomicMin claim,
          owner-bucket counters) -- the measured MI355X baseline
  td      load-balanced top-down (edge-balanced work list, bitmap frontier)
  bu      bottom-up parent search every level
  do      direction-optimising (Beamer alpha/beta switch between td and bu)
  simple  vertex-centric status-array scan (the reference's dead multiBfs)
  scan    atomic-free queue build: relax / count / prefix-scan / assign (the
          reference's driver-API "scan" pipeline, bfs.cu:706-781)
"""
from .bfs import BFS, BFSResult, MODES  # noqa: F401

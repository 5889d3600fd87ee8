"""Streaming-bandwidth probe: copy and 4-in/1-out shapes at several sizes."""
import sys
sys.path.insert(0, '.')
from hpcclassmultigridproject_amd import _lib
for nin in (1, 4):
    for mb in (256, 1024, 2048):
        print(nin, mb, round(_lib.stream_bandwidth(mb << 20, nin, 10), 1), flush=True)

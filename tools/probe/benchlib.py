"""python tools/probe/benchlib.py LIB.so [bench args]: bench.py against another build."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import syncr_amd
syncr_amd.library_path = os.path.abspath(sys.argv[1])
import bench
bench.main(sys.argv[2:])

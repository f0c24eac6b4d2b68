import sys, subprocess
subprocess.check_call([sys.executable, "/root/repo/tools/patches/split.py", sys.argv[1], "leafy"])

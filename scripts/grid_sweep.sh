for g in 1 2 3; do echo "== WG/CU $g"; ERAY_FRAME_WG_PER_CU=$g timeout -k 10 100 python scripts/diag_render.py 2>&1 | grep -v amdgpu.ids; done

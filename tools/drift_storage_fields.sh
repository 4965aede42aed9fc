mkdir -p gpurun_out/r06h
tools/gpu_steps.sh \
  r06h/vel 300 python3 tools/f32_drift.py --storage-fields surge,sway,yaw_rate --out gpurun_out/r06h/vel.json --- \
  r06h/shaft 300 python3 tools/f32_drift.py --storage-fields shaft_speed,heading_prev --out gpurun_out/r06h/shaft.json --- \
  r06h/pose 300 python3 tools/f32_drift.py --storage-fields north,east,yaw --out gpurun_out/r06h/pose.json --- \
  r06h/ints 300 python3 tools/f32_drift.py --storage-fields ship_speed_i,shaft_speed_i,heading_i,e_ct_int --out gpurun_out/r06h/ints.json

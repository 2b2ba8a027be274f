cd $GRAFT_REPO_ROOT
for nl in "" "obs_i8,masks,term,trunc,status" "obs_i32,obs_f32,rewards" "obs_i32,obs_i8,obs_f32,masks,rewards,term,trunc,status"; do
  NULL_OUTS="$nl" timeout -k 10 60 python scripts/diag_time.py 4096 2>&1 | grep -v amdgpu.ids || exit 1
done

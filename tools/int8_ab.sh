for lib in ab/old.so "" ab/old.so ""; do
  SPEF_LIB=$lib timeout -k 10 120 python bench.py --dtype int8 --no-cpu-baseline > gpurun_out/i8.json 2>/dev/null && python -c "import json;d=json.load(open('gpurun_out/i8.json'));print('int8', '${lib:-new}', d['value'])"
done

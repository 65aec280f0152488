import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
idx = [i for i,r in enumerate(rows) if 'adamw' in r['Kernel_Name']]
a, b = idx[-3], idx[-2]
for r in rows[a+1:b+1]:
    n = r['Kernel_Name']
    if 'conv_gemm' in n or 'wgrad_reduce' in n:
        d = (int(r['End_Timestamp']) - int(r['Start_Timestamp']))/1e3
        tag = n.split('conv_gemm_kernelILi')[1][:40] if 'conv' in n else 'reduce'
        print(f"{d:8.1f}us grid={int(r['Grid_Size_X'])//int(r['Workgroup_Size_X'])},{r['Grid_Size_Y']} wg={r['Workgroup_Size_X']} vgpr={r['VGPR_Count']} {tag}")

// Exhaustive check that the kernels' u16 millimetre -> metres conversion, q = m*0.001 with one FMA
// correction, equals NumPy's astype(float)/1000. for every m in [0, 65535].
// gcc -O2 -ffp-contract=off tools/check_depth_conversion.c -lm && ./a.out
#include <stdio.h>
#include <math.h>
int main(){ int bad1=0,bad2=0; double c=0.001;
 for(int m=0;m<65536;m++){ double ref=(double)m/1000.0; double q=(double)m*c; if(q!=ref)bad1++;
   double r=fma(-q,1000.0,(double)m); double q2=fma(r,c,q); if(q2!=ref)bad2++; }
 printf("mul-only mismatches %d, one-correction mismatches %d\n",bad1,bad2); return 0;}

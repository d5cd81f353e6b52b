// CPU check of move_cell_f32_fast (csrc/lnw_device.h) against the exact float32
// move path (double sin / cos, float rounding): 4e7 rows, uniform, dyadic (ties
// likely), wide-range and whole-degree rows.  gcc -O2 -ffp-contract=off
// tools/move_cell_check.c -lm && ./a.out  ->  'mismatches 0'
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
static const double PY_PI=3.141592653589793, RAD2DEG=180.0/3.141592653589793;
static void ref(int px,int py,int speed,float a2,float a3,int*nx,int*ny){
 float course=(float)(2.0*PY_PI)*a2; float dist=(float)speed*a3; double deg=(double)course*RAD2DEG;
 double s=sin(deg),c=cos(deg); float dx=(float)c*dist, dy=(float)s*dist; float fx=(float)px+dx, fy=(float)py+dy;
 *nx=(int)rintf(fx); *ny=(int)rintf(fy);}
static int fast(int px,int py,int speed,float a2,float a3,int*nx,int*ny){
 float course=(float)(2.0*PY_PI)*a2; float dist=(float)speed*a3; double deg=(double)course*RAD2DEG;
 if(!(fabs(deg)<1.0e5)||!(fabsf(dist)<=4.0f))return 0;
 double k=rint(deg*6.36619772367581382433e-01); double rd=fma(-k,1.57079632673412561417e+00,deg); rd=fma(-k,6.07710050650619224932e-11,rd);
 float r=(float)rd, z=r*r;
 float sr=r+r*z*(-1.6666667e-1f+z*(8.3333333e-3f+z*(-1.9841270e-4f+z*2.7557319e-6f)));
 float cr=1.0f-0.5f*z+z*z*(4.1666668e-2f+z*(-1.3888889e-3f+z*2.4801587e-5f));
 int n=(int)k&3; float s=n==0?sr:n==1?cr:n==2?-sr:-cr; float c=n==0?cr:n==1?-sr:n==2?-cr:sr;
 float fx=(float)px+c*dist, fy=(float)py+s*dist; if(!(fabsf(fx)<256.f&&fabsf(fy)<256.f))return 0;
 float rx=rintf(fx), ry=rintf(fy);
 if(fabsf(fabsf(fx-rx)-0.5f)<4e-5f||fabsf(fabsf(fy-ry)-0.5f)<4e-5f)return 0;
 *nx=(int)rx;*ny=(int)ry;return 1;}
int main(){ long n=0,ok=0,bad=0; srand(3);
 for(long i=0;i<40000000;i++){ int px=rand()%200, py=rand()%200, sp=2+(rand()&1);
  float a2,a3; int m=i%4;
  if(m==0){a2=(float)rand()/RAND_MAX; a3=(float)rand()/RAND_MAX;}
  else if(m==1){a2=(float)((rand()%4096)/4096.0); a3=(float)((rand()%8)/8.0);}   /* dyadic: ties likely */
  else if(m==2){a2=(float)(((double)rand()/RAND_MAX-0.5)*20); a3=(float)((double)rand()/RAND_MAX*1.4);}
  else {a2=(float)((rand()%360)/360.0); a3=1.0f;}
  int rx,ry,fx,fy; ref(px,py,sp,a2,a3,&rx,&ry); n++;
  if(fast(px,py,sp,a2,a3,&fx,&fy)){ok++; if(fx!=rx||fy!=ry){bad++; if(bad<5)printf("bad %d %d %d %.9g %.9g\n",px,py,sp,a2,a3);}}}
 printf("n %ld fast %ld (%.6f) mismatches %ld\n",n,ok,(double)ok/n,bad);}
